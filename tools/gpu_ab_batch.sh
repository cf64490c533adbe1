# Parameterised A/B of library builds on one box (replaces round 5's one-off tools/gpu_r05_*.sh).
#   LIBS    "name=path ..."  builds to compare; an empty path is the tree's libmgdp.so
#   CONFIGS "env:B ..."      batched workloads for tools/probe_batch.py
#   TESTS   "tests/... ..."  GPU tests run on every non-default build first (optional)
#   REPS    alternation rounds (default 2), SOLVES / PREPS probe_batch's --solves / --reps
#   TAG     output directory under gpurun_out/
# Output: gpurun_out/$TAG/ab.jsonl (one probe_batch line per build x config x round) and a summary.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab_batch}
mkdir -p $OUT
for spec in $LIBS; do
  name=${spec%%=*}; path=${spec#*=}
  if [ -n "$path" ] && [ -n "$TESTS" ]; then
    MGDP_LIB=$path timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread $TESTS \
      > $OUT/pytest_$name.log 2>&1 || { tail -40 $OUT/pytest_$name.log; echo "tests failed on $name"; exit 1; }
    echo "$name: $(tail -1 $OUT/pytest_$name.log)"
  fi
done
P="python3 -u tools/probe_batch.py --solves ${SOLVES:-5} --reps ${PREPS:-3}"
for rep in $(seq 1 ${REPS:-2}); do
  for spec in $LIBS; do
    name=${spec%%=*}; path=${spec#*=}
    for cfg in $CONFIGS; do
      env=${cfg%%:*}; B=${cfg#*:}
      timeout -k 10 300 env MGDP_LIB=$path $P --tag $name --env $env --B $B >> $OUT/ab.jsonl 2>> $OUT/ab.err \
        || { tail -20 $OUT/ab.err; echo "probe failed: $name $env $B"; exit 1; }
    done
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d = json.loads(l)
    print('%-8s %-34s %6d %9.2f us %9.2f kern %.4g upd/s' % (d['tag'], d['env'], d['B'], d['us_per_solve'], d['kernel_us'], d['updates_per_s']))
" | tee $OUT/summary.txt
echo "all ok"
