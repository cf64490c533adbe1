# Step kernel with nontemporal obs stores (MGDP_STEP_NT=1) / + window loads (=3) vs default, A/B twice,
# 2^20 and 65536 DoorKey-16 envs, plus the step tests on the NT=3 build.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/step_nt
mkdir -p $OUT
MGDP_LIB=$PWD/exp/libmgdp_nt3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_step.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
for lib in minigrid_dynamicprogramming_amd/libmgdp.so exp/libmgdp_nt1.so exp/libmgdp_nt3.so; do
for w in step_doorkey16x1m step_doorkey16x65536; do
n=$(basename $lib .so)
MGDP_LIB=$PWD/$lib timeout -k 10 120 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu > $OUT/${n}_${w}_$rep.json 2>/dev/null || { echo "$n $w failed"; exit 1; }
python -c "import json; d=json.load(open('$OUT/${n}_${w}_$rep.json')); r=d['roofline']; print('$n $w', '%.4g'%d['value'], '%.1f us'%r['avg_launch_us'], 'frac %.3f'%r['frac'])"
done
done
done
