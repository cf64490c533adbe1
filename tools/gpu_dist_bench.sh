# Rehearse bench.py's N > 1 path on a 1-GPU box: `python bench.py --gpus 2` starts its own two ranks
# (no torchrun on the command line), both pinned to device 0 (MGDP_BENCH_DEVICE), gloo for the
# collectives (MGDP_BENCH_BACKEND; RCCL refuses two ranks per GPU).  The driver's multi-GPU runs use
# RCCL, one GPU per rank.  TAG names the run (copy gpurun_out/$TAG to profiles/$TAG).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-distbench}
mkdir -p $OUT
run() { name=$1; shift
  timeout -k 10 400 env MGDP_BENCH_DEVICE=0 MGDP_BENCH_BACKEND=gloo python bench.py --gpus 2 "$@" --no-cpu --no-hbm > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; tail -20 $OUT/$name.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1]); print('$name', d['n_gpus'], '%.4g'%d['value'], '%.1f us'%(d['ms_per_step']*1e3), {k: ('%.4g'%b['value'], b['parallelism'], b['roofline']['traffic']) for k, b in d.get('sharded', {}).items()})"; }
run default --steps 20 --warmup 5
# the driver's own launcher line for N > 1 (torchrun, rendezvous on 127.0.0.1)
timeout -k 10 400 env MGDP_BENCH_DEVICE=0 MGDP_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29000 + RANDOM % 1000)) bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --no-hbm > $OUT/torchrun.json 2> $OUT/torchrun.err || { echo "torchrun failed"; tail -20 $OUT/torchrun.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/torchrun.json').read().strip().splitlines()[-1]); print('torchrun', d['n_gpus'], '%.4g'%d['value'], '%.1f us'%(d['ms_per_step']*1e3))"
run fourrooms1 --workload fourrooms1 --steps 50 --warmup 5
echo all ok
