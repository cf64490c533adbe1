# Delayed stop test for the served lone grid (fused_lone_xyd3, MGDP_LONE3): lone-grid test suites,
# then an A/B of the default bench (driver command) and fourrooms1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-lone3}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_vi.py tests/test_gpu_serve_grids.py tests/test_gpu_rollout.py tests/test_gpu_options.py tests/test_gpu_env_api.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
for l3 in 1 0; do
MGDP_LONE3=$l3 timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-hbm > $OUT/l${l3}_s20_$rep.json 2> $OUT/l${l3}_s20_$rep.err || { echo "bench failed"; tail $OUT/l${l3}_s20_$rep.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/l${l3}_s20_$rep.json')); print('lone3=$l3 s20', '%.4g'%d['value'], '%.3f us'%(d['ms_per_step']*1e3), 'f64 %.4g'%d['f64']['value'])"
MGDP_LONE3=$l3 timeout -k 10 120 python bench.py --gpus 1 --steps 200 --warmup 5 --no-cpu --no-hbm --no-f64 > $OUT/l${l3}_s200_$rep.json 2> $OUT/l${l3}_s200_$rep.err || { echo "bench failed"; exit 1; }
python -c "import json; d=json.load(open('$OUT/l${l3}_s200_$rep.json')); print('lone3=$l3 s200', '%.4g'%d['value'], '%.3f us'%(d['ms_per_step']*1e3))"
MGDP_LONE3=$l3 timeout -k 10 120 python bench.py --workload fourrooms1 --steps 200 --warmup 20 --no-cpu --no-hbm --no-f64 > $OUT/l${l3}_fr1_$rep.json 2> $OUT/l${l3}_fr1_$rep.err || { echo "bench fr1 failed"; exit 1; }
python -c "import json; d=json.load(open('$OUT/l${l3}_fr1_$rep.json')); print('lone3=$l3 fourrooms1', '%.4g'%d['value'], '%.3f us'%(d['ms_per_step']*1e3))"
done
done
echo "all ok"
