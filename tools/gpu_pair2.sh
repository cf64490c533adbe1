# Adjacent-pair XYD fused variant (fused_pair_xyd, MGDP_PAIR2): VI test suites, then the batched
# XYD workloads against the previous two-cells-per-thread path (MGDP_PAIR2=0).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pair2}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_vi.py tests/test_gpu_fullsize.py tests/test_gpu_options.py tests/test_gpu_rollout.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for p in 1 0; do
for w in empty16x65536 lava65536 fourrooms4096; do
MGDP_PAIR2=$p timeout -k 10 120 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu --no-hbm --no-f64 > $OUT/p${p}_$w.json 2> $OUT/p${p}_$w.err || { echo "$p $w failed"; tail $OUT/p${p}_$w.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/p${p}_$w.json')); print('pair2=$p $w', '%.4g'%d['value'], d['roofline']['avg_launch_us'])"
done
done
for w in empty16x65536 lava65536; do
timeout -k 10 120 python bench.py --workload $w --dtype f64 --steps 5 --warmup 2 --no-cpu --no-hbm > $OUT/f64_$w.json 2> $OUT/f64_$w.err || { echo "f64 $w failed"; exit 1; }
python -c "import json; d=json.load(open('$OUT/f64_$w.json')); print('f64 $w', '%.4g'%d['value'], d['roofline']['avg_launch_us'])"
done
echo "all ok"
