# Per-rank work of an N-GPU sharded run, measured on one GPU: MGDP_BENCH_SHARD_OF=N makes the one
# rank solve rank 0's shard of the N-way split of lava65536 / doorkey65536 (8192 grids at N = 8),
# directly and through the sharded device protocol over a one-rank RCCL group (MGDP_BENCH_FORCE_DIST,
# torchrun).  What it leaves out of an N-GPU run: the all-reduce's xGMI latency at N > 1 (its
# one-rank device time is in `collectives`) and the max over ranks of unequal shards.
# TAG names the run (copy gpurun_out/$TAG to profiles/$TAG).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-shard}
mkdir -p $OUT
summ() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['config']['grids_per_gpu'], 'grids', '%.4g'%d['value'], '%.1f us/solve'%(d['ms_per_step']*1e3), 'launches/solve %.2f'%(1/r['solves_per_launch']), '%.1f us/launch'%r['avg_launch_us'], d['config'].get('parallelism'), d.get('collectives'))"; }
for n in ${SHARDS:-1 2 4 8}; do
for w in lava65536 doorkey65536; do
  timeout -k 10 300 env MGDP_BENCH_SHARD_OF=$n python bench.py --workload $w --steps 40 --warmup 5 --no-cpu --no-hbm --no-f64 > $OUT/direct_${w}_of$n.json 2> $OUT/direct_${w}_of$n.err || { echo "direct $w of $n failed"; tail $OUT/direct_${w}_of$n.err; exit 1; }
  summ $OUT/direct_${w}_of$n.json direct_${w}_of$n
  timeout -k 10 300 env MGDP_BENCH_SHARD_OF=$n MGDP_BENCH_FORCE_DIST=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29000 + RANDOM % 1000)) \
    bench.py --workload $w --steps 40 --warmup 5 --no-cpu --no-hbm > $OUT/nccl1_${w}_of$n.json 2> $OUT/nccl1_${w}_of$n.err || { echo "nccl1 $w of $n failed"; tail $OUT/nccl1_${w}_of$n.err; exit 1; }
  summ $OUT/nccl1_${w}_of$n.json nccl1_${w}_of$n
done
done
echo "all ok"
