# Round-2 pass c: the stripped soa fused variant under the VI tests, then the bench region
# broken down per solve (MGDP_BENCH_STAMPS) at 20 and 200 steps.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02c
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_vi.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2 3; do
MGDP_BENCH_STAMPS=1 timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-hbm > $OUT/bench_s20_$i.json 2> $OUT/bench_s20_$i.err || { echo "bench failed"; tail $OUT/bench_s20_$i.err; exit 1; }
done
MGDP_BENCH_STAMPS=1 timeout -k 10 120 python bench.py --gpus 1 --steps 200 --warmup 5 --no-cpu --no-hbm > $OUT/bench_s200.json 2> $OUT/bench_s200.err || { echo "bench failed"; exit 1; }
for w in doorkey65536 lava65536 empty16x65536 fourrooms4096; do
timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu --no-hbm --no-f64 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo "bench $w failed"; tail $OUT/bench_$w.err; exit 1; }
done
echo "all ok"
