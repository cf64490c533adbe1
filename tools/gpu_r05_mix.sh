# Round 5: (1) the full GPU suite after the epoch-tagged host publication (one PCIe write latency per
# result instead of two) and the in-launch reduction for any batch size; (2) A/B of mixed wave counts
# (MGDP_MIX=1: the learned order's long grids on two waves) and of the reduction rule (MGDP_GK=1 any
# B vs 2 resident only) with probe_batch -> ab.jsonl; (3) the 8-way LavaS11N5 shard direct vs the
# library communicator, with and without the mixed launch.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_mix}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_mix.py > $OUT/pytest_mix.log 2>&1 || { tail -40 $OUT/pytest_mix.log; echo "mix tests failed"; exit 1; }
tail -1 $OUT/pytest_mix.log
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu --ignore=tests/test_gpu_mix.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; echo "tests failed"; exit 1; }
tail -1 $OUT/pytest.log
fi
[ -n "$ONLY_TESTS" ] && { echo "all ok"; exit 0; }
P="python3 -u tools/probe_batch.py --solves 10 --reps 3"
run() { tag=$1; shift; kv=(); while [[ "$1" == *=* ]]; do kv+=("$1"); shift; done; timeout -k 10 150 env "${kv[@]}" $P --tag $tag "$@" >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "probe $tag failed"; tail -5 $OUT/ab.err; exit 1; }; }
LAVA=MiniGrid-LavaCrossingS11N5-v0
for rep in 1 2; do
  for B in 8192 2048 512; do
    run mix0 MGDP_MIX=0 --env $LAVA --B $B || exit 1
    for f in 0.5 0.75 0.9; do run mix1_f$f MGDP_MIX=1 MGDP_MIX_FRAC=$f --env $LAVA --B $B || exit 1; done
  done
  for wl in "$LAVA 65536" "MiniGrid-FourRooms-v0 4096" "MiniGrid-Empty-16x16-v0 65536"; do set -- $wl
    run mix0_gk1 MGDP_MIX=0 --env $1 --B $2 || exit 1
    run mix0_gk2 MGDP_MIX=0 MGDP_GK=2 --env $1 --B $2 || exit 1
    run mix1_f0.75 MGDP_MIX=1 MGDP_MIX_FRAC=0.75 --env $1 --B $2 || exit 1
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print('%-12s %-30s %6d %9.2f us %9.2f kern %.4g upd/s k %d x %.3f' % (d['tag'], d['env'], d['B'], d['us_per_solve'], d['kernel_us'], d['updates_per_s'], d['sweeps'], d['executed_frac']))"
summ() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['config']['grids_per_gpu'], 'grids', '%.4g'%d['value'], '%.1f us/solve'%(d['ms_per_step']*1e3), '%.1f us/launch'%r['avg_launch_us'], d['config'].get('parallelism'), d.get('collectives'))"; }
for mix in 0 1; do
  timeout -k 10 300 env MGDP_MIX=$mix MGDP_BENCH_SHARD_OF=8 python bench.py --workload lava65536 --steps 40 --warmup 5 --no-cpu --no-hbm --no-f64 > $OUT/direct_mix$mix.json 2> $OUT/direct_mix$mix.err || { echo "direct mix$mix failed"; tail $OUT/direct_mix$mix.err; exit 1; }
  summ $OUT/direct_mix$mix.json direct_mix$mix
  timeout -k 10 300 env MGDP_MIX=$mix MGDP_BENCH_SHARD_OF=8 MGDP_BENCH_FORCE_DIST=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29000 + RANDOM % 1000)) \
    bench.py --workload lava65536 --steps 40 --warmup 5 --no-cpu --no-hbm --no-f64 > $OUT/lib_mix$mix.json 2> $OUT/lib_mix$mix.err || { echo "lib mix$mix failed"; tail $OUT/lib_mix$mix.err; exit 1; }
  summ $OUT/lib_mix$mix.json lib_mix$mix
done
echo "all ok"
