# Round-2 pass h: env-API conformance tests on the GPU-backed env; the step kernel past the MALL
# (2^20 DoorKey-16 envs) next to 65536; rocprofv3 kernel stats of the driver's default bench
# command; PMC HBM traffic passes (served lone grid, step 1M).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02h
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_env_api.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_env_api.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_env_api.log; exit 1; }
tail -2 $OUT/pytest_env_api.log
for w in step_doorkey16x65536 step_doorkey16x1m; do
timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --cpu-budget 3 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo "bench $w failed"; tail $OUT/bench_$w.err; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/rocprof_default -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $OUT/rocprof_default_bench.json 2> $OUT/rocprof_default.err || { echo "rocprof failed"; tail $OUT/rocprof_default.err; exit 1; }
prof() { name=$1; ctr=$2; shift 2
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace -T -d $OUT/pmc/${name}_${ctr} -o run --output-format csv -- python3 bench.py "$@" --no-cpu --no-hbm --no-f64 > $OUT/pmc_${name}_${ctr}.log 2>&1 || { echo "$name $ctr failed"; exit 1; }; }
for c in FETCH_SIZE WRITE_SIZE; do
  prof empty16 $c --steps 20 --warmup 0
  prof step_doorkey16x1m $c --workload step_doorkey16x1m --steps 5 --warmup 1
done
echo "all ok"
