# SQ counter passes (kernel trace only) on one bench workload W with extra env E (e.g. MGDP_PAIR2=0).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-sq3}
mkdir -p $OUT
prof() { W=$1; name=$2; shift; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -T -d $OUT/sq_${W}_${name} -o run --output-format csv -- python3 bench.py --workload $W --steps 2 --warmup 1 --no-cpu --no-hbm --no-f64 $BARGS > $OUT/sq_${W}_${name}.log 2>&1 || { echo "$W $name failed"; exit 1; }; }
for W in ${WL:-empty16x65536}; do
prof $W p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU || exit 1
prof $W p2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAVES SQ_ACTIVE_INST_SCA || exit 1
prof $W p3 GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_BRANCH SQ_LDS_DATA_FIFO_FULL SQ_ACTIVE_INST_MISC SQ_BUSY_CU_CYCLES SQ_INST_LEVEL_LDS SQ_LDS_UNALIGNED_STALL || exit 1
done
echo "all ok"
