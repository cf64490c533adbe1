# Round 5: the served lone-grid kernel with the goal reward's max only in the directions where a
# wave faces the goal, vs the build before (ablib/libmgdp_base.so): the served GPU tests, then the
# headline (bench.py, lone Empty-16 only) alternated four times per build.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_sgoal}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread $(ls tests/test_gpu_serve*.py) tests/test_gpu_vi.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; echo "tests failed"; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2 3 4; do
  for lib in base new; do
    L=""; [ $lib = base ] && L=ablib/libmgdp_base.so
    MGDP_LIB=$L MGDP_BENCH_DETAIL=$OUT/${lib}_$rep.json timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-sharded --no-cpu --no-f64 --no-hbm > $OUT/${lib}_${rep}_line.json 2> $OUT/${lib}_$rep.err || { echo "bench $lib failed"; tail $OUT/${lib}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${lib}_$rep.json')); l=d['latency']; print('$lib $rep', '%.3f us'%(d['ms_per_step']*1e3), 'gpu %.3f'%l.get('gpu_solve_us', 0))"
  done
done
echo "all ok"
