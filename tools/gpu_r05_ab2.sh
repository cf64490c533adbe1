# Round 5 A/B: learned dispatch order / priority (MGDP_LEARN_ORDER, MGDP_LEARN_PRIO) on the batched
# BASELINE configs and the 8-way Lava shard; the DoorKey-16 kernels (fused_dk_rows, its 6-wave build in
# ablib/, fused_fast_dk_soa).  GPU tests of the touched paths first.  probe_batch.py lines -> ab.jsonl.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_ab2}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fixedpoint.py -k "not capacity" ${EXTRA_TESTS:-} > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; echo "tests failed"; exit 1; }
MGDP_BAND=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wave2.py tests/test_gpu_fullsize.py tests/test_gpu_fixedpoint.py -k "not capacity" > $OUT/pytest_band.log 2>&1 || { tail -40 $OUT/pytest_band.log; echo "band tests failed"; exit 1; }
tail -2 $OUT/pytest_band.log
tail -2 $OUT/pytest.log
P="python3 -u tools/probe_batch.py --solves 10 --reps 3"
run() { tag=$1; shift; kv=(); while [[ "$1" == *=* ]]; do kv+=("$1"); shift; done; timeout -k 10 150 env "${kv[@]}" $P --tag $tag "$@" >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "probe $tag failed"; tail -5 $OUT/ab.err; exit 1; }; }
for rep in 1 2; do
  for lo in "1 1" "0 0" "1 0"; do set -- $lo
    for wl in "MiniGrid-LavaCrossingS11N5-v0 8192" "MiniGrid-LavaCrossingS11N5-v0 65536" "MiniGrid-FourRooms-v0 4096" "MiniGrid-DoorKey-16x16-v0 65536"; do set -- $lo $wl
      run "order$1_prio$2" MGDP_LEARN_ORDER=$1 MGDP_LEARN_PRIO=$2 --env $3 --B $4 || exit 1
    done
  done
  run dkrows0_learn1 MGDP_DK_ROWS=0 --env MiniGrid-DoorKey-16x16-v0 --B 65536 || exit 1
  run dkrows0_learn0 MGDP_DK_ROWS=0 MGDP_LEARN_ORDER=0 MGDP_LEARN_PRIO=0 --env MiniGrid-DoorKey-16x16-v0 --B 65536 || exit 1
  for wl in "MiniGrid-FourRooms-v0 4096" "MiniGrid-LavaCrossingS11N5-v0 65536" "MiniGrid-LavaCrossingS11N5-v0 8192" "MiniGrid-Empty-16x16-v0 65536"; do set -- $wl
    run band1_learn1 MGDP_BAND=1 --env $1 --B $2 || exit 1
    run band1_learn0 MGDP_BAND=1 MGDP_LEARN_ORDER=0 MGDP_LEARN_PRIO=0 --env $1 --B $2 || exit 1
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print('%-16s %-32s %6d %9.2f us %9.2f kern %.4g upd/s k %d x %.3f' % (d['tag'], d['env'], d['B'], d['us_per_solve'], d['kernel_us'], d['updates_per_s'], d['sweeps'], d['executed_frac']))"
echo all ok
