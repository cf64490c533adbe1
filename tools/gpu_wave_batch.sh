# Measurement: batched XYD grids on the one-wave path (no workgroup barrier per sweep) vs the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/wave_batch
mkdir -p $OUT
for cfg in "MGDP_WAVE_BATCH=0" "MGDP_WAVE_BATCH=1 MGDP_WAVE=4" "MGDP_WAVE_BATCH=1 MGDP_WAVE=8"; do
for w in empty16x65536 lava65536 fourrooms4096; do
tag=$(echo $cfg | tr ' =' '__')
env $cfg timeout -k 10 120 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu --no-hbm --no-f64 > $OUT/${tag}_$w.json 2> $OUT/${tag}_$w.err || { echo "$cfg $w failed"; tail $OUT/${tag}_$w.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/${tag}_$w.json')); print('$cfg $w', '%.4g'%d['value'], d['roofline']['avg_launch_us'], d['roofline']['kernel'])"
done
done
MGDP_WAVE_BATCH=1 MGDP_WAVE=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "not doorkey" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
