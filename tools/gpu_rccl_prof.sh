# rocprofv3 kernel stats of the sharded device protocol over a real RCCL communicator at N=1
# (torchrun, one rank, MGDP_BENCH_FORCE_DIST=1): the fused launches and the RCCL all-reduce kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02_rccl_prof
mkdir -p $OUT
MGDP_BENCH_FORCE_DIST=1 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29631 timeout -k 10 300 \
  rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --workload lava65536 --steps 5 --warmup 2 --no-cpu --no-hbm > $OUT/bench.json 2> $OUT/bench.err || { echo "rocprof failed"; tail $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4g'%d['value'], '%.1f us/step'%(d['ms_per_step']*1e3), d['config'].get('parallelism'), d.get('collectives'))"
f=$(find $OUT/prof -name 'run_kernel_stats.csv' | head -1); cut -c1-160 $f
echo "all ok"
