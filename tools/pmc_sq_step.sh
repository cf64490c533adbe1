# SQ counter passes on the batched step kernel (kernel trace only; counters in their own passes).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-sqstep}
mkdir -p $OUT
W=${W:-step_doorkey16x65536}
prof() { name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace -T -d $OUT/${W}_${name} -o run --output-format csv -- python3 bench.py --workload $W --steps 5 --warmup 1 --no-cpu > $OUT/${W}_${name}.log 2>&1 || { echo "$name failed"; exit 1; }; }
prof p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU
prof p2 SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAVES SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM
prof p3 GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_BRANCH SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LEVEL_WAVES SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM
echo sq ok
