# (Measured, not kept: MGDP_STEP_ALIAS / MGDP_STEP_WPE are no longer in envs.hip; the record of profiles/r02_step_alias/.)
# Step kernel: window aliased inside the obs tile (default build) vs separate window (libmgdp_a0,
# -DMGDP_STEP_ALIAS=0) vs aliased + waves_per_eu 8 (libmgdp_w8, 19 VGPRs spilled): step parity tests
# on the default and w8 builds, then the step benches alternating twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02_step_alias
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_env_api.py tests/test_gpu_rollout.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_default.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_default.log; exit 1; }
tail -1 $OUT/pytest_default.log
MGDP_LIB=$PWD/tools/libmgdp_w8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_step.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_w8.log 2>&1 || { echo "pytest w8 failed"; tail -40 $OUT/pytest_w8.log; exit 1; }
tail -1 $OUT/pytest_w8.log
for rep in 1 2; do
for lib in minigrid_dynamicprogramming_amd/libmgdp.so tools/libmgdp_a0.so tools/libmgdp_w8.so; do
n=$(basename $lib .so)
for w in step_doorkey16x1m step_doorkey16x65536 step_fourrooms65536; do
MGDP_LIB=$PWD/$lib timeout -k 10 120 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu > $OUT/${n}_${w}_$rep.json 2> $OUT/${n}_${w}_$rep.err || { echo "$lib $w failed"; tail $OUT/${n}_${w}_$rep.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/${n}_${w}_$rep.json')); r=d['roofline']; print('$n $w', '%.4g'%d['value'], '%.2f us'%r['avg_launch_us'], 'frac %.3f'%r['frac'])"
done
done
done
echo "all ok"
