# Round-2 pass d: served distinct grids (new grid per request) + VI suites, then the default bench
# (rehearsed edges) at 20 and 200 steps with per-solve stamps, and the fourrooms1 workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02d
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_serve_grids.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_serve.log 2>&1 || { echo "pytest serve failed"; tail -40 $OUT/pytest_serve.log; exit 1; }
tail -2 $OUT/pytest_serve.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_vi.py tests/test_gpu_fullsize.py tests/test_gpu_options.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do
MGDP_BENCH_STAMPS=1 timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-hbm > $OUT/bench_s20_$i.json 2> $OUT/bench_s20_$i.err || { echo "bench failed"; tail $OUT/bench_s20_$i.err; exit 1; }
done
MGDP_BENCH_STAMPS=1 timeout -k 10 120 python bench.py --gpus 1 --steps 200 --warmup 5 --no-cpu --no-hbm > $OUT/bench_s200.json 2> $OUT/bench_s200.err || { echo "bench failed"; exit 1; }
MGDP_BENCH_STAMPS=1 timeout -k 10 200 python bench.py --workload fourrooms1 --steps 200 --warmup 20 --cpu-budget 4 --no-hbm > $OUT/bench_fourrooms1.json 2> $OUT/bench_fourrooms1.err || { echo "bench fr1 failed"; tail $OUT/bench_fourrooms1.err; exit 1; }
MGDP_PERSISTENT=0 timeout -k 10 200 python bench.py --workload fourrooms1 --steps 200 --warmup 20 --no-cpu --no-hbm --no-f64 > $OUT/bench_fourrooms1_nopersist.json 2> $OUT/bench_fourrooms1_np.err || { echo "bench fr1 np failed"; tail $OUT/bench_fourrooms1_np.err; exit 1; }
echo "all ok"
