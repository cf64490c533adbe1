# Round 6 evidence on the final build: the full GPU suite and smoke, the driver's bench command (x2),
# its rocprofv3 kernel stats, and the line at 200 steps.  TAG names the run (gpurun_out/$TAG).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06_final}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
for i in 1 2; do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { tail $OUT/bench_$i.err; exit 1; }
  tail -c 2500 $OUT/bench_$i.json
  echo
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/rocprof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $OUT/rocprof_bench.json 2> $OUT/rocprof_bench.err || { tail $OUT/rocprof_bench.err; exit 1; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 5 --no-cpu --no-hbm --no-f64 > $OUT/bench200.json 2> $OUT/bench200.err || { tail $OUT/bench200.err; exit 1; }
tail -c 600 $OUT/bench200.json
