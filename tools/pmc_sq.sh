# SQ counter passes on the batched fused (M=fused) or HBM sweep (M=sweep) kernel (kernel trace only; counters in their own passes).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/sq
mkdir -p $OUT
W=${W:-empty16x65536}
M=${M:-fused}
prof() { name=$1; shift
  timeout -k 10 600 rocprofv3 --pmc "$@" --kernel-trace -T -d $OUT/${W}_${M}_${name} -o run --output-format csv -- python3 bench.py --workload $W --method $M --steps 2 --warmup 1 --no-cpu --no-hbm > $OUT/${W}_${M}_${name}.log 2>&1 || { echo "$name failed"; exit 1; }; }
prof p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU
prof p2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAVES SQ_ACTIVE_INST_SCA
prof p3 GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_BRANCH SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LEVEL_WAVES SQ_INST_LEVEL_LDS
echo sq ok
