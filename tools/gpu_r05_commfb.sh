# Round 5: bench.py's communicator choice at N > 1 -- the library's communicator, or, when
# mgdp_comm_create fails on any rank (rehearsed with MGDP_BENCH_LIB_COMM_FAIL=<rank>), the
# torch.distributed protocol on every rank: one rank on one GPU (MGDP_BENCH_FORCE_DIST=1), the 8-way
# LavaS11N5 shard both ways.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_commfb}
mkdir -p $OUT
for fail in none 0; do
  timeout -k 10 300 env MGDP_BENCH_LIB_COMM_FAIL=$fail MGDP_BENCH_SHARD_OF=8 MGDP_BENCH_FORCE_DIST=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29000 + RANDOM % 1000)) \
    bench.py --workload lava65536 --steps 20 --warmup 5 --no-cpu --no-hbm --no-f64 > $OUT/lib_fail_$fail.json 2> $OUT/lib_fail_$fail.err || { echo "run failed"; tail $OUT/lib_fail_$fail.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/lib_fail_$fail.json').read().strip().splitlines()[-1]); print('fail=$fail', '%.4g'%d['value'], '%.1f us/solve'%(d['ms_per_step']*1e3), d.get('collectives'))"
  grep -h "communicator unavailable" $OUT/lib_fail_$fail.err || true
done
echo "all ok"
