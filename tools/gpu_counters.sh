# Hardware counters of the kernels the bench line prices (TAG names the run; then
#   python tools/pmc_parse.py gpurun_out/$TAG profiles/pmc_traffic.json
#   python tools/sq_counters_json.py gpurun_out/$TAG profiles/sq_counters.json
# and copy gpurun_out/$TAG to profiles/$TAG):
#  * HBM traffic: FETCH_SIZE and WRITE_SIZE in separate passes (kernel trace only; MI355X_MICROARCH.md
#    HBM section: 2 * FETCH_SIZE + WRITE_SIZE per launch on gfx950);
#  * SQ issue / LDS / wait counters of the batched fused kernel in three passes per workload.
# WL overrides the batched workloads (default: the four BASELINE-sized batches).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-counters}
mkdir -p $OUT
prof() { name=$1; ctr=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -T -d $OUT/${name}_${ctr} -o run --output-format csv -- python3 bench.py "$@" --no-cpu --no-hbm --no-f64 --no-sharded > $OUT/${name}_${ctr}.log 2>&1 || { echo "$name $ctr failed"; exit 1; }; }
for c in FETCH_SIZE WRITE_SIZE; do
  prof empty16 $c --steps 20 --warmup 0
  prof empty16x65536_sweep $c --workload empty16x65536 --method sweep --steps 2 --warmup 1
  for W in ${WL:-empty16x65536 lava65536 fourrooms4096 doorkey65536}; do
    prof ${W}_fused $c --workload $W --method fused --steps 2 --warmup 1
  done
done
sq() { W=$1; name=$2; shift; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -T -d $OUT/sq_${W}_${name} -o run --output-format csv -- python3 bench.py --workload $W --steps 2 --warmup 1 --no-cpu --no-hbm --no-f64 > $OUT/sq_${W}_${name}.log 2>&1 || { echo "$W $name failed"; exit 1; }; }
for W in ${WL:-empty16x65536 lava65536 fourrooms4096 doorkey65536}; do
  sq $W p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU || exit 1
  sq $W p2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAVES SQ_ACTIVE_INST_SCA || exit 1
  sq $W p3 GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_BRANCH SQ_LDS_DATA_FIFO_FULL SQ_ACTIVE_INST_MISC SQ_BUSY_CU_CYCLES SQ_INST_LEVEL_LDS SQ_LDS_UNALIGNED_STALL || exit 1
done
echo "all ok"
