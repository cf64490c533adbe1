# Round-2 pass b: lone-grid teardown probe (default host wait vs active wait), then SQ counter
# passes on the batched fused kernel (Empty-16 x 65536, DoorKey-16 x 65536).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02b
mkdir -p $OUT
timeout -k 10 120 python tools/probe_teardown.py > $OUT/teardown_default.json 2> $OUT/teardown.err || { echo "probe failed"; tail $OUT/teardown.err; exit 1; }
timeout -k 10 120 python tools/probe_teardown.py --timing > $OUT/teardown_default_timing.json 2>> $OUT/teardown.err || { echo "probe t failed"; exit 1; }
ROC_ACTIVE_WAIT_TIMEOUT=1000 timeout -k 10 120 python tools/probe_teardown.py > $OUT/teardown_active1000.json 2>> $OUT/teardown.err || { echo "probe a failed"; exit 1; }
prof() { W=$1; name=$2; shift; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -T -d $OUT/sq_${W}_${name} -o run --output-format csv -- python3 bench.py --workload $W --steps 2 --warmup 1 --no-cpu --no-hbm --no-f64 > $OUT/sq_${W}_${name}.log 2>&1 || { echo "$W $name failed"; exit 1; }; }
for W in empty16x65536 doorkey65536; do
prof $W p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU || exit 1
prof $W p2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAVES SQ_ACTIVE_INST_SCA || exit 1
prof $W p3 GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_BRANCH SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_INST_LEVEL_LDS SQ_LEVEL_WAVES || exit 1
prof $W p4 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_ACTIVE_INST_MISC SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 || exit 1
done
echo "all ok"
