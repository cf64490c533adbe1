# Step-kernel pass: parity (step + rollout + options tests), step benches, rocprofv3 kernel stats
# of the default step bench (its average must agree with the bench's event timing).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-step}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_rollout.py tests/test_gpu_options.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_step.log 2>&1 || { echo pytest failed; tail -30 $OUT/pytest_step.log; exit 1; }
for w in step_doorkey16x65536 step_fourrooms65536 step_lava65536; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --cpu-budget 10 > $OUT/$w.json 2> $OUT/$w.err || { echo "$w failed"; exit 1; }
  timeout -k 10 300 env MGDP_STEP_GROUP=1 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu > $OUT/${w}_g1.json 2> $OUT/${w}_g1.err || { echo "$w g1 failed"; exit 1; }
  timeout -k 10 300 env MGDP_STEP_GROUP=4 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu > $OUT/${w}_g4.json 2> $OUT/${w}_g4.err || { echo "$w g4 failed"; exit 1; }
  timeout -k 10 300 env MGDP_STEP_GROUP=8 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu > $OUT/${w}_g8.json 2> $OUT/${w}_g8.err || { echo "$w g8 failed"; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_step -o run --output-format csv -- python3 bench.py --workload step_doorkey16x65536 --steps 20 --warmup 3 --no-cpu > $OUT/prof_step.log 2>&1 || { echo "rocprof step failed"; exit 1; }
echo all ok
