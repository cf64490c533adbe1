# Round 5: where the 8-way LavaS11N5 shard's time goes.  (1) probe_batch over batch sizes 64..8192 (the
# longest grid's sweep chain alone vs at full residency), (2) the sharded solve through the library's
# communicator under rocprofv3 --kernel-trace (tools/gpu_shard_prof.sh: direct, one-rank lib path,
# and its kernel trace).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_lat}
mkdir -p $OUT
for B in 64 512 2048 4096 8192 16384; do
  timeout -k 10 150 python3 -u tools/probe_batch.py --env MiniGrid-LavaCrossingS11N5-v0 --B $B --solves 10 --reps 3 --tag lava$B >> $OUT/lat.jsonl 2>> $OUT/lat.err || { echo "probe $B failed"; exit 1; }
done
python3 -c "
import json
for l in open('$OUT/lat.jsonl'):
    d=json.loads(l); print('%-10s %6d %9.2f us %9.2f kern k %d x %.3f' % (d['tag'], d['B'], d['us_per_solve'], d['kernel_us'], d['sweeps'], d['executed_frac']))"
TAG=${TAG:-r05_lat}/prof WORKLOADS=lava65536 bash tools/gpu_shard_prof.sh || exit 1
echo all ok
