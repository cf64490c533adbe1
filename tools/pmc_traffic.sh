# HBM traffic per launch from PMC counters (separate passes per MI355X_MICROARCH.md: FETCH_SIZE and
# WRITE_SIZE cannot share a pass).  Kernel trace/stats only -- no runtime/sys trace with --pmc.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
prof() { name=$1; ctr=$2; shift 2
  timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-trace -T -d $OUT/${name}_${ctr} -o run --output-format csv -- python3 bench.py "$@" --no-cpu --no-hbm --no-f64 > $OUT/${name}_${ctr}.log 2>&1 || { echo "$name $ctr failed"; exit 1; }; }
for c in FETCH_SIZE WRITE_SIZE; do
  prof empty16 $c --steps 20 --warmup 0
  prof empty16x65536_sweep $c --workload empty16x65536 --method sweep --steps 2 --warmup 1
  prof empty16x65536_fused $c --workload empty16x65536 --method fused --steps 2 --warmup 1
  prof doorkey65536_fused $c --workload doorkey65536 --method fused --steps 1 --warmup 0
done
echo pmc ok
