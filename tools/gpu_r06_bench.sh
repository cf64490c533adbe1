# Round 6: the headline bench (the driver's command shape) alternating builds / knobs:
# KNOBS="name=ENV=VAL,ENV2=VAL2 name2=..." (default: MGDP_SERVE_PAIR 1 vs 0), REPS rounds, STEPS timed solves.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06_bench}
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread $TESTS > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
for rep in $(seq 1 ${REPS:-3}); do
  for spec in ${KNOBS:-pair1=MGDP_SERVE_PAIR=1 pair0=MGDP_SERVE_PAIR=0}; do
    name=${spec%%=*}; envs=${spec#*=}
    timeout -k 10 120 env ${envs//,/ } python3 bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu --no-hbm --no-f64 ${BENCH_ARGS} > $OUT/bench_${name}_$rep.json 2> $OUT/bench_${name}_$rep.err || { tail $OUT/bench_${name}_$rep.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/bench_${name}_$rep.json').read().strip().splitlines()[-1]); print('$name', d['value'], round(d['ms_per_step']*1e3, 3), 'us', d.get('lat_us'))"
  done
done
