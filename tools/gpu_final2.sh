# Evidence after the nontemporal sweep change: full GPU suite, smoke, default bench line + rocprof
# stats, sweep-method benches, and PMC traffic of the sweep kernel (separate counter passes).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/final2
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_default -o run --output-format csv -- python3 bench.py --warmup 0 --no-cpu --no-hbm > $OUT/prof_default.log 2>&1 || { echo "rocprof failed"; exit 1; }
for w in empty16x65536 doorkey65536; do
  timeout -k 10 600 python bench.py --workload $w --method sweep --steps 5 --warmup 1 --no-cpu > $OUT/bench_${w}_sweep.json 2> $OUT/bench_${w}_sweep.err || { echo "bench $w failed"; exit 1; }
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -T -d $OUT/pmc/sweep_$c -o run --output-format csv -- python3 bench.py --workload empty16x65536 --method sweep --steps 2 --warmup 1 --no-cpu --no-hbm > $OUT/pmc_sweep_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
echo "all ok"
