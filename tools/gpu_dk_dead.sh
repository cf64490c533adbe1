# Batched DoorKey A/B: DoorKey GPU tests on the default build, then the default libmgdp.so vs the
# builds in $B_LIBS (default abl/libmgdp_nodead.so, -DMGDP_DK_DEAD=0): run_to(69) timing + the doorkey65536 bench, twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r03_dk_dead}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_vi.py tests/test_gpu_resume.py tests/test_gpu_options.py -k "doorkey or DoorKey or dk" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for rep in 1 2; do
for lib in minigrid_dynamicprogramming_amd/libmgdp.so ${B_LIBS:-abl/libmgdp_nodead.so}; do
n=$(basename $lib .so)
MGDP_LIB=$PWD/$lib timeout -k 10 120 python tools/probe_dk_runto.py doorkey65536 69 > $OUT/runto_${n}_$rep.json 2>$OUT/runto_${n}_$rep.err || { tail $OUT/runto_${n}_$rep.err; exit 1; }
cat $OUT/runto_${n}_$rep.json
MGDP_LIB=$PWD/$lib timeout -k 10 120 python bench.py --workload doorkey65536 --steps 5 --warmup 2 --no-cpu --no-hbm --no-f64 > $OUT/${n}_$rep.json 2> $OUT/${n}_$rep.err || { tail $OUT/${n}_$rep.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/${n}_$rep.json')); print('$n', '%.4g'%d['value'], '%.1f'%d['roofline']['avg_launch_us'])"
done
done
