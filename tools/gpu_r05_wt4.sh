# Round 5: write-through exit stores also in the sharded protocol's run_local launches of a resident
# batch (Geo::wt) vs the build before them (ablib/libmgdp_base.so = plain stores everywhere): the XYD
# and protocol GPU tests, then the 8-way LavaS11N5 rank-0 shard direct and through the library
# communicator (bench.py, no per-launch events in the region), alternating builds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_wt4}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wave2.py tests/test_gpu_fixedpoint.py tests/test_gpu_distributed.py tests/test_gpu_fullsize.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; echo "tests failed"; exit 1; }
tail -1 $OUT/pytest.log
summ() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', '%.4g'%d['value'], '%.1f us/solve'%(d['ms_per_step']*1e3), '%.1f us/launch'%r['avg_launch_us'], d['config'].get('parallelism'))"; }
for rep in 1 2; do
  for lib in base new; do
    L=""; [ $lib = base ] && L=ablib/libmgdp_base.so
    timeout -k 10 300 env MGDP_LIB=$L MGDP_BENCH_SPLIT_EVENTS=1 MGDP_BENCH_SHARD_OF=8 python3 bench.py --workload lava65536 --steps 40 --warmup 5 --no-cpu --no-hbm --no-f64 > $OUT/direct_${lib}_$rep.json 2> $OUT/direct_${lib}_$rep.err || { echo "direct failed"; tail $OUT/direct_${lib}_$rep.err; exit 1; }
    summ $OUT/direct_${lib}_$rep.json direct_$lib
    timeout -k 10 300 env MGDP_LIB=$L MGDP_BENCH_SPLIT_EVENTS=1 MGDP_BENCH_SHARD_OF=8 MGDP_BENCH_FORCE_DIST=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29000 + RANDOM % 1000)) \
      bench.py --workload lava65536 --steps 40 --warmup 5 --no-cpu --no-hbm --no-f64 > $OUT/lib_${lib}_$rep.json 2> $OUT/lib_${lib}_$rep.err || { echo "lib failed"; tail $OUT/lib_${lib}_$rep.err; exit 1; }
    summ $OUT/lib_${lib}_$rep.json lib_$lib
  done
done
echo "all ok"
