# The batch server's GPU-side solve time vs the launch's kernel time (tools/probe_bserve.py), for
# library builds LIBS "name=path ..." (empty path = the tree's) and CONFIGS "env:B ...".
# Output: gpurun_out/$TAG/probe.jsonl
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06_bserve_probe}
mkdir -p $OUT
CONFIGS=${CONFIGS:-"MiniGrid-LavaCrossingS11N5-v0:8192 MiniGrid-LavaCrossingS11N5-v0:4096 MiniGrid-LavaCrossingS11N5-v0:2048 MiniGrid-FourRooms-v0:4096"}
LIBS=${LIBS:-"main="}
for rep in $(seq 1 ${REPS:-2}); do
  for spec in $LIBS; do
    name=${spec%%=*}; path=${spec#*=}
    for cfg in $CONFIGS; do
      env=${cfg%%:*}; B=${cfg#*:}
      timeout -k 10 300 env MGDP_LIB=$path python3 -u tools/probe_bserve.py --env $env --B $B --tag $name $PROBE_ARGS >> $OUT/probe.jsonl 2>> $OUT/probe.err \
        || { tail -20 $OUT/probe.err; echo "probe failed: $name $env $B"; exit 1; }
    done
  done
done
cat $OUT/probe.jsonl
echo "all ok"
