# VI quick pass: GPU VI/options parity, the lone-grid C-ABI latency probe, the headline bench line
# (no CPU baseline) and the batched fused benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-viq}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_vi.py tests/test_gpu_options.py tests/test_gpu_rollout.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo pytest failed; tail -30 $OUT/pytest.log; exit 1; }
timeout -k 10 120 ./tools/probe_serve default > $OUT/probe_serve.json 2> $OUT/probe_serve.err || { echo probe failed; exit 1; }
timeout -k 10 300 python bench.py --no-cpu --no-hbm > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo bench failed; exit 1; }
for w in empty16x65536 doorkey65536 lava65536 fourrooms4096; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 1 --no-cpu > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo "bench $w failed"; exit 1; }
done
timeout -k 10 300 env MGDP_DK_1T=1 python bench.py --workload doorkey65536 --steps 5 --warmup 1 --no-cpu > $OUT/bench_doorkey65536_dk1t.json 2> /dev/null || { echo "bench dk1t failed"; exit 1; }
for w in empty16x65536 doorkey65536 lava65536 fourrooms4096; do
  timeout -k 10 300 env MGDP_CPT=1 python bench.py --workload $w --steps 5 --warmup 1 --no-cpu > $OUT/bench_${w}_cpt1.json 2> /dev/null || { echo "bench $w cpt1 failed"; exit 1; }
  timeout -k 10 300 env MGDP_CPT=4 python bench.py --workload $w --steps 5 --warmup 1 --no-cpu > $OUT/bench_${w}_cpt4.json 2> /dev/null || { echo "bench $w cpt4 failed"; exit 1; }
done
echo all ok
