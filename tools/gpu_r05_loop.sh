# Round 5: the sweep loops with the stop test at the end of the deciding sweep (fused_wave2_xyd,
# fused_dk_rows: no loop-carried copy of V_{k-1}, 10-36 fewer VGPR moves per sweep).  Full GPU suite,
# then A/B against the previous build (ablib/libmgdp_r05a.so, MGDP_LIB) with probe_batch -> ab.jsonl,
# then the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_loop}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; echo "tests failed"; exit 1; }
tail -1 $OUT/pytest.log
fi
P="python3 -u tools/probe_batch.py --solves 10 --reps 3"
run() { tag=$1; shift; kv=(); while [[ "$1" == *=* ]]; do kv+=("$1"); shift; done; timeout -k 10 150 env "${kv[@]}" $P --tag $tag "$@" >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "probe $tag failed"; tail -5 $OUT/ab.err; exit 1; }; }
for rep in 1 2; do
  for wl in "MiniGrid-LavaCrossingS11N5-v0 65536" "MiniGrid-LavaCrossingS11N5-v0 8192" "MiniGrid-FourRooms-v0 4096" "MiniGrid-Empty-16x16-v0 65536" "MiniGrid-DoorKey-16x16-v0 65536"; do set -- $wl
    run base MGDP_LIB=ablib/libmgdp_r05a.so MGDP_GK=2 --env $1 --B $2 || exit 1
    run new MGDP_GK=2 --env $1 --B $2 || exit 1
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print('%-6s %-30s %6d %9.2f us %9.2f kern %.4g upd/s k %d x %.3f' % (d['tag'], d['env'], d['B'], d['us_per_solve'], d['kernel_us'], d['updates_per_s'], d['sweeps'], d['executed_frac']))"
MGDP_BENCH_DETAIL=$OUT/bench_detail.json timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo "all ok"
