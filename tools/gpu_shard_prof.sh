# Where the sharded protocol's time goes at an 8-way shard, on one GPU: the one-rank RCCL rehearsal
# (MGDP_BENCH_FORCE_DIST=1, MGDP_BENCH_SHARD_OF=8: rank 0's shard of the 8-way split) run directly
# under rocprofv3 --kernel-trace (the rank's env is set here, no torchrun hop), beside the direct
# solve of the same shard.  TAG names the run (copy gpurun_out/$TAG to profiles/$TAG).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-shard_prof}
mkdir -p $OUT
summ() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['config']['grids_per_gpu'], 'grids', '%.4g'%d['value'], '%.1f us/solve'%(d['ms_per_step']*1e3), 'launches/solve %.2f'%(1/r['solves_per_launch']), '%.1f us/launch'%r['avg_launch_us'], d.get('collectives'), d.get('executed_rank0'))"; }
for w in ${WORKLOADS:-lava65536 doorkey65536}; do
  timeout -k 10 300 env MGDP_BENCH_SHARD_OF=8 MGDP_BENCH_SPLIT_EVENTS=1 python bench.py --workload $w --steps 40 --warmup 5 --no-cpu --no-hbm --no-f64 > $OUT/direct_$w.json 2> $OUT/direct_$w.err || { echo "direct $w failed"; tail $OUT/direct_$w.err; exit 1; }
  summ $OUT/direct_$w.json direct_$w
  export MGDP_BENCH_SHARD_OF=8 MGDP_BENCH_FORCE_DIST=1 MGDP_BENCH_SPLIT_EVENTS=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29000 + RANDOM % 1000))
  timeout -k 10 300 python bench.py --workload $w --steps 40 --warmup 5 --no-cpu --no-hbm > $OUT/nccl1_$w.json 2> $OUT/nccl1_$w.err || { echo "nccl1 $w failed"; tail $OUT/nccl1_$w.err; exit 1; }
  summ $OUT/nccl1_$w.json nccl1_$w
  export MASTER_PORT=$((29000 + RANDOM % 1000))
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 40 --warmup 5 --no-cpu --no-hbm > $OUT/prof_$w.json 2> $OUT/prof_$w.err || { echo "rocprof $w failed"; tail $OUT/prof_$w.err; exit 1; }
  summ $OUT/prof_$w.json prof_$w
  unset MGDP_BENCH_SHARD_OF MGDP_BENCH_FORCE_DIST MGDP_BENCH_SPLIT_EVENTS WORLD_SIZE RANK LOCAL_RANK MASTER_ADDR MASTER_PORT
done
echo "all ok"
