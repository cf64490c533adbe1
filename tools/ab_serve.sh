# A/B of lone-grid (served Empty-16x16) builds: ALT names the alternative library (an MGDP_BUILD_OUT
# build with MGDP_EXTRA_FLAGS), TAG the run.  Served-path GPU tests on ALT first, then the headline
# bench (no blocks, no CPU legs) alternating default / ALT, REPS times.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-ab_serve}
mkdir -p $OUT
MGDP_LIB=$ALT timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_serve_ew.py tests/test_gpu_serve_grids.py tests/test_gpu_resume.py -m gpu > $OUT/pytest_alt.log 2>&1 || { echo "alt tests failed"; tail -30 $OUT/pytest_alt.log; exit 1; }
tail -1 $OUT/pytest_alt.log
for rep in $(seq ${REPS:-3}); do
  for lib in minigrid_dynamicprogramming_amd/libmgdp.so $ALT; do
    n=$(basename $(dirname $lib))_$rep
    MGDP_LIB=$lib timeout -k 10 200 python bench.py --gpus 1 --steps ${STEPS:-200} --warmup 5 --no-cpu --no-hbm --no-sharded --no-f64 > $OUT/$n.json 2> $OUT/$n.err || { echo "bench $n failed"; tail $OUT/$n.err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); l=d['latency']; print('$n', '%.4g'%d['value'], '%.3f us'%(d['ms_per_step']*1e3), 'gpu %.3f'%l['gpu_solve_us'], 'sweeps', d['sweeps'])"
  done
done
echo all ok
