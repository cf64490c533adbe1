# (Measured and dropped: the one-launch solve is no longer in the library -- polling one launch-wide word
#  serialised the grids, 104 vs 46 us at 64 FourRooms grids; record of profiles/r02_gsync/.)
# One-launch batched solve (launch-wide stop in fused_wave2_xyd): its GPU tests (incl. the abort
# fallback) and the wave2 / full-size suites, then FourRooms x 4096 (the batch is resident at once)
# with the path on and off, alternating twice; then the whole GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02_gsync
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_gsync.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gsync.log 2>&1 || { echo "gsync tests failed"; tail -40 $OUT/pytest_gsync.log; exit 1; }
tail -1 $OUT/pytest_gsync.log
for rep in 1 2; do
for gs in 1 0; do
for w in fourrooms4096; do
MGDP_GSYNC=$gs timeout -k 10 120 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu --no-hbm --no-f64 > $OUT/gs${gs}_${w}_$rep.json 2> $OUT/gs${gs}_${w}_$rep.err || { echo "$w gs$gs failed"; tail $OUT/gs${gs}_${w}_$rep.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/gs${gs}_${w}_$rep.json')); r=d['roofline']; print('gs$gs $w', '%.4g'%d['value'], '%.1f us/solve'%(d['ms_per_step']*1e3), 'launch %.1f us x %d'%(r['avg_launch_us'], r['launches']), d['sweeps'])"
done
done
done
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
echo "all ok"
