# Lone-grid replicas under a process group at world 1: none / gloo / nccl, alternating twice, to find
# what a torch.distributed process group costs the resident server's host-polled solves.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02_dist_penalty
mkdir -p $OUT
for rep in 1 2; do
for mode in none gloo nccl; do
if [ $mode = none ]; then envs=""; else envs="MGDP_BENCH_FORCE_DIST=1 MGDP_BENCH_BACKEND=$mode"; fi
env $envs timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2962$rep \
    bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-hbm --no-f64 > $OUT/${mode}_$rep.json 2> $OUT/${mode}_$rep.err || { echo "$mode failed"; tail $OUT/${mode}_$rep.err; exit 1; }
tail -1 $OUT/${mode}_$rep.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$mode $rep', '%.4g'%d['value'], '%.2f us/step'%(d['ms_per_step']*1e3))"
done
done
echo "all ok"
