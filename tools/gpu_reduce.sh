# Vectorised launch reduction (vi_reduce_kernel, B > 512): full GPU suite, the batched benches, and
# rocprofv3 stats of Lava x 65536 (the reduce kernel's own duration).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02_reduce}
mkdir -p $OUT
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for w in lava65536 empty16x65536 fourrooms4096 doorkey65536; do
timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu --no-hbm --no-f64 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo "bench $w failed"; tail $OUT/bench_$w.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_$w.json')); r=d['roofline']; print('$w', '%.4g'%d['value'], '%.1f us/step'%(d['ms_per_step']*1e3), 'launch %.1f us'%r['avg_launch_us'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --workload lava65536 --steps 10 --warmup 2 --no-cpu --no-hbm --no-f64 > $OUT/rocprof_lava.json 2> $OUT/rocprof_lava.err || { echo "rocprof failed"; exit 1; }
f=$(find $OUT/prof -name 'run_kernel_stats.csv' | head -1); grep -i "reduce\|Name" $f | cut -c1-170
echo "all ok"
