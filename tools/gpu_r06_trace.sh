# Round 6: served lone-grid latency split, pair loop (MGDP_SERVE_PAIR=1) vs single (0): the served-path
# tests, C-ABI solve latency (probe_serve) and, on the trace build (ablib/trace/libmgdp.so,
# -DMGDP_SERVE_TRACE), the GPU-side request seen -> publish time and shader clock; then the headline
# bench alternating the two (200 timed solves).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06_trace}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_serve_ew.py tests/test_gpu_serve_grids.py tests/test_gpu_vi.py tests/test_gpu_resume.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for pair in 1 0; do
    MGDP_SERVE_PAIR=$pair timeout -k 10 120 ./tools/probe_serve pair$pair >> $OUT/serve.json 2>> $OUT/serve.err || { echo "probe failed"; exit 1; }
    MGDP_SERVE_PAIR=$pair LD_LIBRARY_PATH=ablib/trace timeout -k 10 120 ./tools/probe_serve trace_pair$pair >> $OUT/trace.json 2> $OUT/trace_p$pair.err || { echo "trace probe failed"; exit 1; }
    grep "serve trace" $OUT/trace_p$pair.err | tail -1
  done
done
cat $OUT/serve.json
for rep in 1 2; do
  for pair in 1 0; do
    timeout -k 10 120 env MGDP_SERVE_PAIR=$pair python3 bench.py --steps 200 --warmup 5 --no-cpu --no-hbm --no-f64 > $OUT/bench_p${pair}_$rep.json 2> $OUT/bench_p${pair}_$rep.err || { tail $OUT/bench_p${pair}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/bench_p${pair}_$rep.json').read().strip().splitlines()[-1]); print('pair=$pair', d['value'], round(d['ms_per_step']*1e3, 3), 'us', d.get('lat_us'))"
  done
done
