# SURVEY 8(f) rows 1-2 measured: step / generator side benches, rocprof stats of the step kernel,
# and the lone-grid latency breakdown through the C ABI (tools/probe_serve, built on the CPU host).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-side}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_rollout.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_step.log 2>&1 || { echo pytest failed; tail -30 $OUT/pytest_step.log; exit 1; }
timeout -k 10 120 ./tools/probe_serve default > $OUT/probe_serve.json 2> $OUT/probe_serve.err || { echo probe_serve failed; exit 1; }
timeout -k 10 120 env MGDP_PERSISTENT=0 ./tools/probe_serve nopersist >> $OUT/probe_serve.json 2>> $OUT/probe_serve.err || { echo probe_serve2 failed; exit 1; }
for w in step_doorkey16x65536 step_fourrooms65536 step_lava65536; do
  timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --cpu-budget 10 > $OUT/$w.json 2> $OUT/$w.err || { echo "$w failed"; exit 1; }
done
for w in gen_lava65536 gen_fourrooms65536 gen_doorkey16x65536; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 1 --cpu-budget 10 > $OUT/$w.json 2> $OUT/$w.err || { echo "$w failed"; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_step -o run --output-format csv -- python3 bench.py --workload step_doorkey16x65536 --steps 20 --warmup 3 --no-cpu > $OUT/prof_step.log 2>&1 || { echo "rocprof step failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_gen -o run --output-format csv -- python3 bench.py --workload gen_lava65536 --steps 5 --warmup 1 --no-cpu > $OUT/prof_gen.log 2>&1 || { echo "rocprof gen failed"; exit 1; }
echo all ok
