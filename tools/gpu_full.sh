# Full GPU pass: tests, default bench, rocprof kernel stats, side workloads.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/prof_default -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu > gpurun_out/prof_default.log 2>&1 && \
for w in empty16x65536 fourrooms4096 lava65536 doorkey65536; do
  for m in fused sweep; do
    timeout -k 10 600 python bench.py --workload $w --method $m --steps 5 --warmup 1 --no-cpu --no-hbm > gpurun_out/bench_${w}_${m}.json 2> gpurun_out/bench_${w}_${m}.err || exit 1
  done
done
echo "exit $?"
