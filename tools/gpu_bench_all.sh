# GPU pass: parity tests, default bench, per-workload benches (fused/sweep x cell/sa), rocprof stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_default -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu --no-hbm > $OUT/prof_default.log 2>&1 || exit 1
for w in empty16 empty16x65536 fourrooms4096 lava65536 doorkey65536; do
  for m in fused sweep; do
    for p in cell sa; do
      timeout -k 10 600 python bench.py --workload $w --method $m --mapping $p --steps 5 --warmup 1 --no-cpu --no-hbm > $OUT/bench_${w}_${m}_${p}.json 2> $OUT/bench_${w}_${m}_${p}.err || exit 1
    done
  done
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_R_sweep -o run --output-format csv -- python3 bench.py --workload empty16x65536 --method sweep --steps 5 --warmup 1 --no-cpu --no-hbm > $OUT/prof_R.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_R_fused -o run --output-format csv -- python3 bench.py --workload empty16x65536 --method fused --steps 5 --warmup 1 --no-cpu --no-hbm > $OUT/prof_R2.log 2>&1 || exit 1
echo "all ok"
