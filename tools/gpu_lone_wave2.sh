# The lone served grid on one wave (MGDP_LONE_WAVE2=1, fused_wave2_xyd in vi_serve_kernel) vs the
# default 4-wave server: serve / VI tests under the knob, then default bench and fourrooms1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-lone_wave2}
mkdir -p $OUT
MGDP_LONE_WAVE2=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_serve_grids.py tests/test_gpu_vi.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for lw in 1 0; do
for i in 1 2; do
MGDP_LONE_WAVE2=$lw timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-hbm > $OUT/lw${lw}_s20_$i.json 2> $OUT/lw${lw}_s20_$i.err || { echo "bench failed"; tail $OUT/lw${lw}_s20_$i.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/lw${lw}_s20_$i.json')); print('lone_wave2=$lw s20', '%.4g'%d['value'], '%.3f us'%(d['ms_per_step']*1e3), 'f64 %.4g'%d['f64']['value'])"
done
MGDP_LONE_WAVE2=$lw timeout -k 10 120 python bench.py --gpus 1 --steps 200 --warmup 5 --no-cpu --no-hbm > $OUT/lw${lw}_s200.json 2> $OUT/lw${lw}_s200.err || { echo "bench failed"; exit 1; }
python -c "import json; d=json.load(open('$OUT/lw${lw}_s200.json')); print('lone_wave2=$lw s200', '%.4g'%d['value'], '%.3f us'%(d['ms_per_step']*1e3), 'f64 %.4g'%d['f64']['value'])"
MGDP_LONE_WAVE2=$lw timeout -k 10 120 python bench.py --workload fourrooms1 --steps 200 --warmup 20 --no-cpu --no-hbm --no-f64 > $OUT/lw${lw}_fr1.json 2> $OUT/lw${lw}_fr1.err || { echo "bench fr1 failed"; exit 1; }
python -c "import json; d=json.load(open('$OUT/lw${lw}_fr1.json')); print('lone_wave2=$lw fourrooms1', '%.4g'%d['value'], '%.3f us'%(d['ms_per_step']*1e3))"
done
echo "all ok"
