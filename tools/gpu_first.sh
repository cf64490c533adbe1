# The driver's bench command FIRST in a fresh lease (per-solve stamps on), then again, then its
# rocprofv3 kernel-trace summary, then the served-grid GPU tests.  TAG names the run; copy
# gpurun_out/$TAG to profiles/$TAG.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-first}
mkdir -p $OUT
for i in ${RUNS:-1 2}; do
MGDP_BENCH_STAMPS=1 MGDP_BENCH_DETAIL=$OUT/bench_${i}_detail.json timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { echo "bench $i failed"; tail $OUT/bench_$i.err; exit 1; }
python -c "
import json; d=json.load(open('$OUT/bench_${i}_detail.json')); print('stdout line chars', len(open('$OUT/bench_$i.json').read())); l=d['latency']; r=d['roofline']
print('bench $i', '%.4g'%d['value'], '%.3f us'%(d['ms_per_step']*1e3), 'f64 %.3f us'%(d['f64']['ms_per_step']*1e3),
      'first %.1f'%l['first_solve_us'], 'primed', l['priming_solves'], l['priming_ms'], 'ms', l['priming_window_medians_us'],
      'clk', l.get('device_clock'), 'launch/solve %.3f'%(r['avg_launch_us']/r['solves_per_launch']))
print({k: ('%.4g'%b['value'], b.get('cpu_baseline',{}).get('value'), b.get('cpu_baseline_all_cores',{}).get('value')) for k, b in {**d.get('batched',{}), **d.get('sharded',{})}.items()})
print('cpu', d['cpu_baseline']['value'], d['cpu_baseline_all_cores']['value'])"
grep stamps $OUT/bench_$i.err | tail -1
done
[ -n "$SKIP_PROF" ] || MGDP_BENCH_DETAIL=$OUT/rocprof_bench.json timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/rocprof_default -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-hbm > $OUT/rocprof_bench_line.json 2> $OUT/rocprof.err || { echo "rocprof failed"; tail $OUT/rocprof.err; exit 1; }
[ -n "$SKIP_PROF" ] || python -c "import json; d=json.load(open('$OUT/rocprof_bench.json')); r=d['roofline']; print('rocprof run', '%.4g'%d['value'], '%.3f us'%(d['ms_per_step']*1e3), 'launch us', r['avg_launch_us'], 'solves', r['solves_per_launch'])"
[ -n "$SKIP_PROF" ] || python tools/rocprof_timed.py $OUT/rocprof_default/run_kernel_trace.csv $OUT/rocprof_bench.json $OUT/rocprof_timed_launch.json > /dev/null
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 $OUT/pytest.log
echo "all ok"
