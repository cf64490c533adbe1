# Round-2 first GPU pass: full GPU suite (with the full-size batched parity tests and the device
# protocol tests), the default bench at --steps 20 and 200 (the headline must not depend on K),
# and a rocprofv3 kernel-trace/stats pass of the default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02a
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
cp gpurun_out/fullsize_sweeps.json $OUT/ 2>/dev/null
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench_s20.json 2> $OUT/bench_s20.err || { echo "bench s20 failed"; tail $OUT/bench_s20.err; exit 1; }
timeout -k 10 600 python bench.py --steps 200 --warmup 20 --no-cpu --no-hbm > $OUT/bench_s200.json 2> $OUT/bench_s200.err || { echo "bench s200 failed"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_default -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-hbm --no-f64 > $OUT/prof_default.log 2>&1 || { echo "rocprof failed"; exit 1; }
echo "all ok"
