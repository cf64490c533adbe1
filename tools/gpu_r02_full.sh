# Round-2 full pass: every GPU test, smoke(), the driver's default bench command, rocprof stats of it.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02_full}
mkdir -p $OUT
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo "bench failed"; tail $OUT/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_default.json')); print('default', '%.4g'%d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('cpu_baseline',{}).get('value'))"
for w in empty16x65536 lava65536 fourrooms4096 doorkey65536 fourrooms1; do
timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 2 --cpu-budget 4 > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo "bench $w failed"; tail $OUT/bench_$w.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_$w.json')); print('$w', '%.4g'%d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline'].get('valu',{}).get('frac'))"
done
echo "all ok"
