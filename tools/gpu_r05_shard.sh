# Round 5: the sharded solve through the library's own RCCL communicator (mgdp_vi_solve_sharded)
# vs the torch.distributed protocol vs the direct solve, on rank 0's shard of an N-way split
# (MGDP_BENCH_SHARD_OF=N, one rank on one GPU; see tools/gpu_shard.sh), plus the distributed GPU tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_shard}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_distributed.py tests/test_gpu_fixedpoint.py ${EXTRA_TESTS:-} > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; echo "tests failed"; exit 1; }
tail -2 $OUT/pytest.log
summ() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['config']['grids_per_gpu'], 'grids', '%.4g'%d['value'], '%.1f us/solve'%(d['ms_per_step']*1e3), 'launches/solve %.2f'%(1/r['solves_per_launch']), '%.1f us/launch'%r['avg_launch_us'], d['config'].get('parallelism'), d.get('collectives'))"; }
for n in ${SHARDS:-8}; do
for w in ${WLS:-lava65536 doorkey65536}; do
  timeout -k 10 300 env MGDP_BENCH_SHARD_OF=$n python bench.py --workload $w --steps 40 --warmup 5 --no-cpu --no-hbm --no-f64 > $OUT/direct_${w}_of$n.json 2> $OUT/direct_${w}_of$n.err || { echo "direct $w of $n failed"; tail $OUT/direct_${w}_of$n.err; exit 1; }
  summ $OUT/direct_${w}_of$n.json direct_${w}_of$n
  for lc in 1 0; do
  timeout -k 10 300 env MGDP_BENCH_LIB_COMM=$lc MGDP_BENCH_SHARD_OF=$n MGDP_BENCH_FORCE_DIST=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29000 + RANDOM % 1000)) \
    bench.py --workload $w --steps 40 --warmup 5 --no-cpu --no-hbm --no-f64 > $OUT/rccl1_lib${lc}_${w}_of$n.json 2> $OUT/rccl1_lib${lc}_${w}_of$n.err || { echo "rccl1 lib$lc $w of $n failed"; tail $OUT/rccl1_lib${lc}_${w}_of$n.err; exit 1; }
  summ $OUT/rccl1_lib${lc}_${w}_of$n.json rccl1_lib${lc}_${w}_of$n
  done
done
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail $OUT/bench_default.err; exit 1; }
tail -c 2100 $OUT/bench_default.json
echo "all ok"
