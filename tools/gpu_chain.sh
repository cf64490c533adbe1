# Chained batched solve (run_local -> run_to with K in device memory, MGDP_CHAIN): VI suites, then
# an on/off A/B of the batched workloads.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-chain}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_vi.py tests/test_gpu_fullsize.py tests/test_gpu_wave2.py tests/test_gpu_options.py tests/test_gpu_serve_grids.py tests/test_gpu_distributed.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
for ch in 1 0; do
for w in fourrooms4096 lava65536 doorkey65536; do
MGDP_CHAIN=$ch timeout -k 10 200 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu --no-hbm --no-f64 > $OUT/c${ch}_${w}_$rep.json 2> $OUT/c${ch}_${w}_$rep.err || { echo "$ch $w failed"; tail $OUT/c${ch}_${w}_$rep.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/c${ch}_${w}_$rep.json')); print('chain=$ch $w', '%.4g'%d['value'], '%.1f us/step'%(d['ms_per_step']*1e3), '%.1f'%d['roofline']['avg_launch_us'])"
done
done
done
echo "all ok"
