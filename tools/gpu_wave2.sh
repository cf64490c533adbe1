# One-wave-per-grid batched XYD (fused_wave2_xyd, MGDP_WAVE2=max cells per lane, 0 = off):
# VI suites for correctness, then the batched XYD workloads in f32 / f64 against MGDP_WAVE2=0.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-wave2}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_vi.py tests/test_gpu_fullsize.py tests/test_gpu_options.py tests/test_gpu_rollout.py tests/test_gpu_distributed.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for dt in f32 f64; do
for w2 in 8 0; do
for w in empty16x65536 lava65536 fourrooms4096; do
MGDP_WAVE2=$w2 timeout -k 10 120 python bench.py --workload $w --dtype $dt --steps 5 --warmup 2 --no-cpu --no-hbm --no-f64 > $OUT/${dt}_w${w2}_$w.json 2> $OUT/${dt}_w${w2}_$w.err || { echo "$dt $w2 $w failed"; tail $OUT/${dt}_w${w2}_$w.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/${dt}_w${w2}_$w.json')); print('$dt wave2<=$w2 $w', '%.4g'%d['value'], '%.1f'%d['roofline']['avg_launch_us'])"
done
done
done
echo "all ok"
