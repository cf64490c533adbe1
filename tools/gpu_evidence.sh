# Round evidence on one build (TAG names the round, e.g. TAG=r03_evidence; copy the result to
# profiles/$TAG): every GPU test, smoke(), the driver's bench command twice and at 200 steps,
# rocprofv3 kernel-trace stats of the driver command, the batched / side workloads.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-evidence}
mkdir -p $OUT
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for i in 1 2; do
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_default_$i.json 2> $OUT/bench_default_$i.err || { echo "bench failed"; tail $OUT/bench_default_$i.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_default_$i.json')); print('default', '%.4g'%d['value'], '%.3f us'%(d['ms_per_step']*1e3), 'f64 %.4g'%d['f64']['value'], 'frac %.4f'%d['roofline']['frac'], {k: '%.4g'%b['value'] for k, b in d.get('sharded', {}).items()})"
done
timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 5 --no-cpu --no-hbm --no-sharded > $OUT/bench_default_s200.json 2> $OUT/bench_default_s200.err || { echo "bench failed"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_default_s200.json')); print('default s200', '%.4g'%d['value'], '%.3f us'%(d['ms_per_step']*1e3))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/rocprof_default -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-hbm --no-sharded > $OUT/rocprof_default_bench.json 2> $OUT/rocprof_default.err || { echo "rocprof failed"; tail $OUT/rocprof_default.err; exit 1; }
for w in empty16x65536 lava65536 fourrooms4096 doorkey65536; do
timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 --cpu-budget 4 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo "bench $w failed"; tail $OUT/bench_$w.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_$w.json')); r=d['roofline']; print('$w', '%.4g'%d['value'], '%.1f us/step'%(d['ms_per_step']*1e3), r['kernel'], 'launches/solve %.1f'%(r['launches']/10), 'valu', r.get('valu',{}).get('frac'), 'hbm', r['frac'], 'f64 %.4g'%d['f64']['value'])"
done
timeout -k 10 300 python bench.py --workload fourrooms1 --steps 200 --warmup 20 --cpu-budget 4 > $OUT/bench_fourrooms1.json 2> $OUT/bench_fourrooms1.err || { echo "bench fr1 failed"; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_fourrooms1.json')); print('fourrooms1', '%.4g'%d['value'], '%.2f us/step'%(d['ms_per_step']*1e3))"
for w in step_doorkey16x1m step_doorkey16x65536 gen_lava65536; do
timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --cpu-budget 3 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo "bench $w failed"; tail $OUT/bench_$w.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_$w.json')); r=d['roofline']; print('$w', '%.4g'%d['value'], d['unit'], '%.1f us'%r['avg_launch_us'], 'frac %.3f'%r['frac'])"
done
echo "all ok"
