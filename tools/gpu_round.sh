# Round-end evidence pass: full GPU parity suite, the default bench line (with CPU baseline and the
# HBM side measurement), rocprofv3 kernel-trace stats of the same default command (HBM side
# measurement off so only the headline kernel's launches are averaged), per-workload benches and
# PMC traffic passes (FETCH_SIZE / WRITE_SIZE in separate passes, kernel trace only).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-round}
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_default -o run --output-format csv -- python3 bench.py --warmup 0 --no-cpu --no-hbm > $OUT/prof_default.log 2>&1 || { echo "rocprof failed"; exit 1; }
for w in empty16x65536 fourrooms4096 lava65536 doorkey65536; do
  timeout -k 10 600 python bench.py --workload $w --steps 5 --warmup 1 --no-cpu > $OUT/bench_${w}.json 2> $OUT/bench_${w}.err || { echo "bench $w failed"; exit 1; }
done
timeout -k 10 600 python bench.py --workload empty16x65536 --method sweep --steps 5 --warmup 1 --no-cpu > $OUT/bench_empty16x65536_sweep.json 2> $OUT/bench_empty16x65536_sweep.err || { echo "bench sweep failed"; exit 1; }
P=$OUT/pmc
mkdir -p $P
prof() { name=$1; ctr=$2; shift 2
  timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-trace -T -d $P/${name}_${ctr} -o run --output-format csv -- python3 bench.py "$@" --no-cpu --no-hbm > $P/${name}_${ctr}.log 2>&1 || { echo "$name $ctr failed"; exit 1; }; }
for c in FETCH_SIZE WRITE_SIZE; do
  prof empty16 $c --steps 20 --warmup 0
  prof empty16x65536_sweep $c --workload empty16x65536 --method sweep --steps 2 --warmup 1
  prof empty16x65536_fused $c --workload empty16x65536 --method fused --steps 2 --warmup 1
  prof doorkey65536_fused $c --workload doorkey65536 --method fused --steps 1 --warmup 0
  prof lava65536_fused $c --workload lava65536 --method fused --steps 1 --warmup 0
  prof fourrooms4096_fused $c --workload fourrooms4096 --method fused --steps 2 --warmup 1
done
echo "all ok"
