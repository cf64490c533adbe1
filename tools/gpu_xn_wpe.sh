# Experiment: the batched two-cells-per-thread XYD fused variant built with amdgpu_waves_per_eu
# 6 / 8 (VGPR cap 80 / 64, with spills) against the default build (95 VGPRs, 5 waves per SIMD).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/xn_wpe
mkdir -p $OUT
for lib in libmgdp.so libmgdp_wpe6.so libmgdp_wpe8.so; do
for w in empty16x65536 lava65536 fourrooms4096; do
MGDP_LIB=$PWD/minigrid_dynamicprogramming_amd/$lib timeout -k 10 120 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu --no-hbm --no-f64 > $OUT/${lib}_$w.json 2> $OUT/${lib}_$w.err || { echo "$lib $w failed"; tail $OUT/${lib}_$w.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/${lib}_$w.json')); print('$lib $w', '%.4g'%d['value'], d['roofline']['avg_launch_us'])"
done
done
MGDP_LIB=$PWD/minigrid_dynamicprogramming_amd/libmgdp_wpe6.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "not doorkey" > $OUT/pytest_wpe6.log 2>&1 || { echo "pytest wpe6 failed"; tail -20 $OUT/pytest_wpe6.log; exit 1; }
tail -1 $OUT/pytest_wpe6.log
