# Round 6: dispatch order from the cells (default, MGDP_ORDER unset) vs round 5's learned order
# (MGDP_ORDER=learned) vs none (off): the order tests, then probe_batch (repeated solves of the same
# grids) alternating the three on the batched BASELINE configs, then the bench's blocks (fresh-grid
# first solves beside the repeated region).  SKIP_TESTS / SKIP_AB skip those parts.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06_order}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fixedpoint.py tests/test_gpu_fullsize.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
if [ -z "$SKIP_AB" ]; then
  P="python3 -u tools/probe_batch.py --solves 5 --reps 3"
  for rep in 1 2; do
    for o in cells learned off; do
      for cfg in MiniGrid-FourRooms-v0:4096 MiniGrid-LavaCrossingS11N5-v0:65536 MiniGrid-DoorKey-16x16-v0:65536; do
        env=${cfg%%:*}; B=${cfg#*:}
        timeout -k 10 300 env MGDP_ORDER=$o $P --tag $o --env $env --B $B >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
      done
    done
  done
  python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d = json.loads(l)
    print('%-8s %-34s %6d %9.2f us %9.2f kern %.4g upd/s' % (d['tag'], d['env'], d['B'], d['us_per_solve'], d['kernel_us'], d['updates_per_s']))
" | tee $OUT/summary.txt
fi
for o in ${ORDERS:-cells learned off}; do
  timeout -k 10 300 env MGDP_ORDER=$o python3 bench.py --steps 20 --warmup 5 --no-cpu --no-hbm --no-f64 > $OUT/bench_$o.json 2> $OUT/bench_$o.err || { tail $OUT/bench_$o.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/bench_$o.json').read().strip().splitlines()[-1]); print('$o', json.dumps(d['configs']))"
done
