# Round 6: the served lone grid on two sweeps per barrier (fused_serve_pair): the served-path GPU tests,
# then the headline bench alternating MGDP_SERVE_PAIR=1 / 0 (200 timed solves each, no CPU / side legs).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06_serve}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_serve_ew.py tests/test_gpu_serve_grids.py tests/test_gpu_vi.py ${EXTRA_TESTS} > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2 3; do
  for pair in 1 0; do
    timeout -k 10 120 env MGDP_SERVE_PAIR=$pair python3 bench.py --steps 200 --warmup 5 --no-cpu --no-hbm --no-f64 > $OUT/bench_p${pair}_$rep.json 2> $OUT/bench_p${pair}_$rep.err || { tail $OUT/bench_p${pair}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/bench_p${pair}_$rep.json').read().strip().splitlines()[-1]); print('pair=$pair', d['value'], d['ms_per_step']*1e3, 'us', d.get('lat_us'), d['roofline'].get('kernel'))"
  done
done
