# bench.py's distributed path on its real backend at N=1: torchrun, one rank, backend nccl (RCCL),
# for the replicated headline and the two sharded configs (MGDP_BENCH_FORCE_DIST=1: process group and
# sharded device protocol at world 1 -- the RCCL K and dV all-reduces run on the library stream).
# on the library stream).  N>1 needs one GPU per rank (the driver's multi-GPU runs).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02_nccl1
mkdir -p $OUT
run() { name=$1; port=$2; shift 2
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port \
    bench.py --gpus 1 "$@" --no-cpu --no-hbm > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail $OUT/$name.err; exit 1; }
  tail -1 $OUT/$name.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', '%.4g'%d['value'], '%.1f us/step'%(d['ms_per_step']*1e3), d['config'].get('parallelism'), d.get('collectives'))"; }
run empty16 29611 --steps 20 --warmup 5
export MGDP_BENCH_FORCE_DIST=1
run empty16_dist 29614 --steps 20 --warmup 5
run lava65536 29612 --workload lava65536 --steps 5 --warmup 2
run doorkey65536 29613 --workload doorkey65536 --steps 3 --warmup 1
echo "all ok"
