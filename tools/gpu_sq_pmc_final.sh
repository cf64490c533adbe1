# SQ counters (3 passes) and HBM traffic (FETCH_SIZE / WRITE_SIZE) of the batched fused kernels as
# built now: Empty-16 x 65536, Lava x 65536, FourRooms x 4096 (wave2), DoorKey-16 x 65536.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=sq_final WL="empty16x65536 lava65536 fourrooms4096" bash tools/pmc_sq3.sh || exit 1
OUT=gpurun_out/pmc_final
mkdir -p $OUT
prof() { name=$1; ctr=$2; shift 2
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace -T -d $OUT/${name}_${ctr} -o run --output-format csv -- python3 bench.py "$@" --no-cpu --no-hbm --no-f64 > $OUT/${name}_${ctr}.log 2>&1 || { echo "$name $ctr failed"; exit 1; }; }
for c in FETCH_SIZE WRITE_SIZE; do
  prof empty16x65536_fused $c --workload empty16x65536 --method fused --steps 2 --warmup 1
  prof lava65536_fused $c --workload lava65536 --method fused --steps 2 --warmup 1
  prof fourrooms4096_fused $c --workload fourrooms4096 --method fused --steps 2 --warmup 1
done
echo "all ok"
