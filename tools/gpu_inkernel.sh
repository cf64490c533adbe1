# In-kernel {k, dV} reduction for larger batches (MGDP_INKERNEL_MAX) vs the separate reduce kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-inkernel}
mkdir -p $OUT
MGDP_INKERNEL_MAX=100000 timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_wave2.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
for m in 512 8192 100000; do
for w in fourrooms4096 lava65536 empty16x65536; do
MGDP_INKERNEL_MAX=$m timeout -k 10 200 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu --no-hbm --no-f64 > $OUT/m${m}_${w}_$rep.json 2> $OUT/m${m}_${w}_$rep.err || { echo "$m $w failed"; tail $OUT/m${m}_${w}_$rep.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/m${m}_${w}_$rep.json')); print('inkernel<=$m $w', '%.4g'%d['value'], '%.1f us/step'%(d['ms_per_step']*1e3), '%.1f'%d['roofline']['avg_launch_us'])"
done
done
done
echo "all ok"
