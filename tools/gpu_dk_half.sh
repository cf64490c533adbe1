# fused_dk_half: DoorKey parity tests, then the doorkey65536 bench with the split on / off.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/dk_half
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_dk_half.py tests/test_gpu_paths.py tests/test_gpu_serve_grids.py -k "dk_half or doorkey" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_vi.py -k "doorkey or maximum" > $OUT/pytest_vi.log 2>&1 || { echo "pytest vi failed"; tail -30 $OUT/pytest_vi.log; exit 1; }
tail -1 $OUT/pytest_vi.log
timeout -k 10 300 python tools/probe_dk_lone.py > $OUT/probe_dk_lone.log 2>&1 || { echo "probe failed"; tail $OUT/probe_dk_lone.log; exit 1; }
cat $OUT/probe_dk_lone.log | head -4
for h in 1 0; do
MGDP_DK_HALF=$h timeout -k 10 300 python bench.py --workload doorkey65536 --steps 10 --warmup 2 --no-cpu > $OUT/bench_h$h.json 2> $OUT/bench_h$h.err || { echo "bench failed"; tail $OUT/bench_h$h.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_h$h.json')); r=d['roofline']; print('half=$h', '%.4g'%d['value'], '%.1f us/step'%(d['ms_per_step']*1e3), r['kernel'], '%.1f us/launch'%r['avg_launch_us'])"
done
for h in 1 0; do
MGDP_DK_HALF=$h timeout -k 10 300 python bench.py --workload doorkey65536 --dtype f64 --steps 5 --warmup 1 --no-cpu > $OUT/bench_f64_h$h.json 2> $OUT/bench_f64_h$h.err || { echo "bench f64 failed"; tail $OUT/bench_f64_h$h.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_f64_h$h.json')); print('f64 half=$h', '%.4g'%d['value'], '%.1f us/step'%(d['ms_per_step']*1e3))"
done
echo "all ok"
