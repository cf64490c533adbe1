# The resident batch server (vi_bserve_kernel): parity tests, then wall per solve with the server
# (MGDP_BSERVE=1, the default) and without it (a launch per solve), alternated REPS times.
# KNOBS "name=ENV=VAL,ENV=VAL ..." (default: on= off=MGDP_BSERVE=0).
# TESTS (default: the batch server's and the batched suites), SKIP_TESTS=1 to skip them.
# Output: gpurun_out/$TAG/{pytest.log, ab.jsonl, summary.txt}
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06_bserve}
mkdir -p $OUT
TESTS=${TESTS:-"tests/test_gpu_bserve.py tests/test_gpu_fixedpoint.py tests/test_gpu_wave2.py tests/test_gpu_distributed.py"}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS > $OUT/pytest.log 2>&1 \
    || { tail -60 $OUT/pytest.log; echo "tests failed"; exit 1; }
  tail -3 $OUT/pytest.log
fi
CONFIGS=${CONFIGS:-"MiniGrid-FourRooms-v0:4096 MiniGrid-LavaCrossingS11N5-v0:8192 MiniGrid-LavaCrossingS11N5-v0:2048 MiniGrid-Empty-16x16-v0:4096"}
KNOBS=${KNOBS:-"on= off=MGDP_BSERVE=0"}
for rep in $(seq 1 ${REPS:-2}); do
  for spec in $KNOBS; do
    name=${spec%%=*}; envs=${spec#*=}
    for cfg in $CONFIGS; do
      env=${cfg%%:*}; B=${cfg#*:}
      timeout -k 10 300 env ${envs//,/ } python3 -u tools/probe_batch.py --solves ${SOLVES:-50} --reps 5 --tag $name \
        --env $env --B $B >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -20 $OUT/ab.err; echo "probe failed: $name $env $B"; exit 1; }
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
