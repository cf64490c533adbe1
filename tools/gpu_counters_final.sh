# Final counters for the batched fused kernels as built: SQ (3 passes) and HBM traffic
# (FETCH_SIZE / WRITE_SIZE), every dispatch counted (chained solves: run_local + run_to).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=sq_final2 WL="empty16x65536 lava65536 fourrooms4096 doorkey65536" bash tools/pmc_sq3.sh || exit 1
OUT=gpurun_out/pmc_final2
mkdir -p $OUT
prof() { name=$1; ctr=$2; shift 2
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace -T -d $OUT/${name}_${ctr} -o run --output-format csv -- python3 bench.py "$@" --no-cpu --no-hbm --no-f64 > $OUT/${name}_${ctr}.log 2>&1 || { echo "$name $ctr failed"; exit 1; }; }
for c in FETCH_SIZE WRITE_SIZE; do
  prof empty16x65536_fused $c --workload empty16x65536 --method fused --steps 2 --warmup 1
  prof lava65536_fused $c --workload lava65536 --method fused --steps 2 --warmup 1
  prof fourrooms4096_fused $c --workload fourrooms4096 --method fused --steps 2 --warmup 1
  prof doorkey65536_fused $c --workload doorkey65536 --method fused --steps 1 --warmup 0
  prof empty16 $c --steps 20 --warmup 0
done
echo "all ok"
