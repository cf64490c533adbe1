# Batched DoorKey-16 x 65536 A/B of library builds: LDS bank-conflict counters (SQ p2 pass) and
# probe_batch timing per build.  LIBS names the builds (default: the product and ablib/*.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-dk_ab}
mkdir -p $OUT
LIBS=${LIBS:-"minigrid_dynamicprogramming_amd/libmgdp.so $(ls ablib/*.so 2>/dev/null)"}
for lib in $LIBS; do
  n=$(basename $lib .so)
  MGDP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU --kernel-trace -T -d $OUT/${n}_p2 -o run --output-format csv -- python3 tools/probe_batch.py --env ${ENV:-MiniGrid-DoorKey-16x16-v0} --B ${B:-65536} --solves 2 --reps 1 --tag $n > $OUT/${n}_p2.log 2>&1 || { echo "sq $n failed"; exit 1; }
done
for rep in 1 2; do
  for lib in $LIBS; do
    MGDP_LIB=$lib timeout -k 10 120 python3 -u tools/probe_batch.py --env ${ENV:-MiniGrid-DoorKey-16x16-v0} --B ${B:-65536} --solves ${SOLVES:-10} --reps 3 --tag $(basename $lib .so) >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "probe $lib failed"; exit 1; }
  done
done
cat $OUT/ab.jsonl
for lib in $LIBS; do python3 tools/sq_summary.py $OUT/$(basename $lib .so) > $OUT/summary_$(basename $lib .so).json || true; done
cat $OUT/summary_*.json
echo all ok
