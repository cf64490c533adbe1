# Round-2 pass e: server exit word (synchronize without a stream drain) + longer priming; serve
# tests, then the default bench at 20 / 200 steps with stamps (x2 each), and fourrooms1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02e
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_serve_grids.py tests/test_gpu_vi.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do
MGDP_BENCH_STAMPS=1 timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-hbm > $OUT/bench_s20_$i.json 2> $OUT/bench_s20_$i.err || { echo "bench failed"; tail $OUT/bench_s20_$i.err; exit 1; }
MGDP_BENCH_STAMPS=1 timeout -k 10 120 python bench.py --gpus 1 --steps 200 --warmup 5 --no-cpu --no-hbm > $OUT/bench_s200_$i.json 2> $OUT/bench_s200_$i.err || { echo "bench failed"; exit 1; }
done
MGDP_BENCH_STAMPS=1 timeout -k 10 200 python bench.py --workload fourrooms1 --steps 200 --warmup 20 --no-cpu --no-hbm > $OUT/bench_fourrooms1.json 2> $OUT/bench_fourrooms1.err || { echo "bench fr1 failed"; tail $OUT/bench_fourrooms1.err; exit 1; }
echo "all ok"
