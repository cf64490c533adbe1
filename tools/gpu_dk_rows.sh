# Round 5: batched DoorKey-16 on fused_dk_rows vs fused_fast_dk_soa (MGDP_DK_ROWS=0), same build.
# 1) the DoorKey GPU tests (new dk_rows file + the existing DoorKey cases), 2) SQ counters (LDS, VALU,
# waits) per variant, 3) probe_batch timing, alternating variants.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-dk_rows}
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dk_rows.py \
  tests/test_gpu_dk_half.py tests/test_gpu_fullsize.py ${EXTRA_TESTS:-} > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; echo "tests failed"; exit 1; }
tail -3 $OUT/pytest.log
for v in 1 0; do
  MGDP_DK_ROWS=$v timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU --kernel-trace -T -d $OUT/rows${v}_p2 -o run --output-format csv -- python3 tools/probe_batch.py --env MiniGrid-DoorKey-16x16-v0 --B 65536 --solves 2 --reps 1 --tag rows$v > $OUT/rows${v}_p2.log 2>&1 || { echo "sq rows$v failed"; exit 1; }
  MGDP_DK_ROWS=$v timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -T -d $OUT/rows${v}_p1 -o run --output-format csv -- python3 tools/probe_batch.py --env MiniGrid-DoorKey-16x16-v0 --B 65536 --solves 2 --reps 1 --tag rows$v > $OUT/rows${v}_p1.log 2>&1 || { echo "sq1 rows$v failed"; exit 1; }
  python3 tools/sq_summary.py $OUT/rows$v > $OUT/summary_rows$v.json || true
done
for rep in 1 2; do
  for v in 1 0; do
    MGDP_DK_ROWS=$v timeout -k 10 120 python3 -u tools/probe_batch.py --env MiniGrid-DoorKey-16x16-v0 --B ${B:-65536} --solves 10 --reps 3 --tag rows$v >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "probe rows$v failed"; exit 1; }
  done
done
cat $OUT/ab.jsonl
cat $OUT/summary_rows*.json
echo all ok
