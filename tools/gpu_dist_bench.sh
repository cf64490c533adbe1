# Rehearse bench.py's N>1 path on a 1-GPU box: 2 ranks pinned to device 0, gloo for the
# collectives (RCCL refuses two ranks per GPU).  The driver's multi-GPU runs use RCCL, one GPU per rank.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/distbench
mkdir -p $OUT
run() { name=$1; port=$2; shift 2
  timeout -k 10 300 env MGDP_BENCH_DEVICE=0 MGDP_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 "$@" --no-cpu --no-hbm > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; exit 1; }; }
run empty16 29511 --steps 20 --warmup 2
run lava65536 29512 --workload lava65536 --steps 3 --warmup 1
run doorkey65536 29513 --workload doorkey65536 --steps 2 --warmup 1
run fourrooms1 29514 --workload fourrooms1 --steps 50 --warmup 5
echo all ok
