# (Variant measured slower and dropped: the MGDP_PAIR_TEST loop is no longer in vi_loops.h; kept as the record of profiles/r02_pairtest/.)
# Stop rule once per pair of sweeps (lone / served XYD grid): full GPU suite on the new build, then
# an A/B against the per-sweep build (tools/libmgdp_pt0.so, -DMGDP_PAIR_TEST=0), alternating twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02_pairtest
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for rep in 1 2; do
for lib in minigrid_dynamicprogramming_amd/libmgdp.so tools/libmgdp_pt0.so; do
n=$(basename $lib .so)
for st in 20 200; do
MGDP_LIB=$PWD/$lib timeout -k 10 120 python bench.py --steps $st --warmup 5 --no-cpu --no-hbm > $OUT/${n}_s${st}_$rep.json 2> $OUT/${n}_s${st}_$rep.err || { echo "$lib bench failed"; tail $OUT/${n}_s${st}_$rep.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/${n}_s${st}_$rep.json')); print('$n s$st', '%.4g'%d['value'], '%.3f us'%(d['ms_per_step']*1e3), 'f64 %.4g'%d['f64']['value'], d['sweeps'])"
done
MGDP_LIB=$PWD/$lib timeout -k 10 120 python bench.py --workload fourrooms1 --steps 200 --warmup 20 --no-cpu --no-hbm > $OUT/${n}_fr1_$rep.json 2> $OUT/${n}_fr1_$rep.err || { echo "$lib fr1 failed"; exit 1; }
python -c "import json; d=json.load(open('$OUT/${n}_fr1_$rep.json')); print('$n fourrooms1', '%.4g'%d['value'], '%.3f us'%(d['ms_per_step']*1e3))"
done
done
echo "all ok"
