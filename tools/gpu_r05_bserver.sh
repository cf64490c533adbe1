# Round 5: tools/probe_batch_server -- request-to-result time of a resident batch (one-wave workgroups
# + the in-launch reduction tree) with a launch per request vs a persistent server that forwards the
# host's request word through a device word (round-6 item 1's design, measured on its skeleton).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_bserver}
mkdir -p $OUT
hipcc -O2 --offload-arch=gfx950 -o $OUT/probe_batch_server tools/probe_batch_server.cpp || { echo "build failed"; exit 1; }
for cfg in ${CFGS:-"8192 0 500 10" "8192 0 500 2" "8192 0 500 40" "4096 0 500 10" "8192 3000 300 10" "256 0 500 10"}; do
  timeout -k 10 60 $OUT/probe_batch_server $cfg >> $OUT/bserver.jsonl 2>> $OUT/bserver.err || { echo "probe $cfg failed"; tail -5 $OUT/bserver.err; cat $OUT/bserver.jsonl; exit 1; }
done
rm -f $OUT/probe_batch_server
cat $OUT/bserver.jsonl
echo "all ok"
