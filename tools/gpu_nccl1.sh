# bench.py's distributed path on its real backend at N = 1: torchrun, one rank, backend nccl (RCCL),
# MGDP_BENCH_FORCE_DIST=1 (process group and the sharded device protocol at world 1: the RCCL
# all-reduce runs on the protocol stream between the shard's launches), against the direct solve of
# the same batch; rocprofv3 kernel stats of the Lava protocol run.  N > 1 needs one GPU per rank
# (the driver's multi-GPU runs).  TAG names the run (copy gpurun_out/$TAG to profiles/$TAG).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-nccl1}
mkdir -p $OUT
summ() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', '%.4g'%d['value'], '%.1f us/solve'%(d['ms_per_step']*1e3), d['config'].get('parallelism'), d.get('collectives'))"; }
for w in lava65536 doorkey65536; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu --no-hbm --no-f64 > $OUT/direct_$w.json 2> $OUT/direct_$w.err || { echo "direct $w failed"; tail $OUT/direct_$w.err; exit 1; }
  summ $OUT/direct_$w.json direct_$w
  timeout -k 10 300 env MGDP_BENCH_FORCE_DIST=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29000 + RANDOM % 1000)) \
    bench.py --workload $w --steps 20 --warmup 3 --no-cpu --no-hbm > $OUT/nccl1_$w.json 2> $OUT/nccl1_$w.err || { echo "nccl1 $w failed"; tail $OUT/nccl1_$w.err; exit 1; }
  summ $OUT/nccl1_$w.json nccl1_$w
done
export MGDP_BENCH_FORCE_DIST=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29000 + RANDOM % 1000))
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --workload lava65536 --steps 20 --warmup 3 --no-cpu --no-hbm > $OUT/prof_lava65536.json 2> $OUT/prof_lava65536.err || { echo "rocprof failed"; tail $OUT/prof_lava65536.err; exit 1; }
echo "all ok"
