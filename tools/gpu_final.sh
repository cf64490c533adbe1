# Final-tree check: full GPU parity suite, smoke, default bench line and its rocprof kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-final}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_default -o run --output-format csv -- python3 bench.py --warmup 0 --no-cpu --no-hbm > $OUT/prof_default.log 2>&1 || { echo "rocprof failed"; exit 1; }
echo "all ok"
