# DoorKey on one wave per grid (fused_wave2_dk, MGDP_DK_WAVE2=max cells per lane): DoorKey VI tests
# under the knob (incl. the full DoorKey-16 x 65536 batch vs the oracle), then the bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-dk_wave2}
mkdir -p $OUT
MGDP_DK_WAVE2=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_vi.py tests/test_gpu_fullsize.py tests/test_gpu_rollout.py -m gpu -x -q --timeout 300 --timeout-method thread -k "doorkey or DoorKey or dk" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for w2 in 4 0; do
MGDP_DK_WAVE2=$w2 timeout -k 10 200 python bench.py --workload doorkey65536 --steps 3 --warmup 1 --no-cpu --no-hbm --no-f64 > $OUT/w${w2}.json 2> $OUT/w${w2}.err || { echo "bench $w2 failed"; tail $OUT/w${w2}.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/w${w2}.json')); print('dk_wave2<=$w2', '%.4g'%d['value'], '%.1f'%d['roofline']['avg_launch_us'])"
done
echo "all ok"
