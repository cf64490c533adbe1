# Round 5: batched DoorKey-16 on fused_dk_rows (KD waves: pickup / unlock targets folded into the
# front value, per-state g): DoorKey GPU tests, probe_batch timing (learned order on / off) and the
# SQ counter passes of the doorkey65536 launch (sq_summary).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_dk}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dk_rows.py tests/test_gpu_dk_half.py tests/test_gpu_fullsize.py ${EXTRA_TESTS:-} > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; echo "tests failed"; exit 1; }
tail -2 $OUT/pytest.log
for rep in 1 2; do
  for lo in 1 0; do
    MGDP_LEARN_ORDER=$lo timeout -k 10 150 python3 -u tools/probe_batch.py --env MiniGrid-DoorKey-16x16-v0 --B 65536 --solves 10 --reps 3 --tag order$lo >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "probe failed"; exit 1; }
  done
done
cat $OUT/ab.jsonl
sq() { name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -T -d $OUT/dk_$name -o run --output-format csv -- python3 tools/probe_batch.py --env MiniGrid-DoorKey-16x16-v0 --B 65536 --solves 2 --reps 1 > $OUT/dk_$name.log 2>&1 || { echo "sq $name failed"; exit 1; }; }
sq p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU || exit 1
sq p2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAVES SQ_ACTIVE_INST_SCA || exit 1
sq p3 GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_BRANCH SQ_LDS_DATA_FIFO_FULL SQ_ACTIVE_INST_MISC SQ_BUSY_CU_CYCLES SQ_INST_LEVEL_LDS SQ_LDS_UNALIGNED_STALL || exit 1
python3 tools/sq_summary.py $OUT/dk > $OUT/summary_doorkey65536.json
cat $OUT/summary_doorkey65536.json
echo all ok
