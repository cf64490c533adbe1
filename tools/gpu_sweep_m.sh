# Sweep-kernel grouping probe: grids staged per workgroup iteration (MGDP_SWEEP_M) x grid size.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-sweepm}
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_gpu_vi.py -x -q > $OUT/pytest_vi.log 2>&1 || { echo pytest failed; exit 1; }
run() { name=$1; shift; timeout -k 10 300 env "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; exit 1; }; }
for m in 1 2 3 4; do for g in 1024 2048 4096; do
  run R_sweep_m${m}_g${g} MGDP_SWEEP_M=$m MGDP_SWEEP_GRID=$g python bench.py --workload empty16x65536 --method sweep --steps 5 --warmup 1 --no-cpu --no-hbm
done; done
for m in 1 2 4; do
  run D_sweep_m${m} MGDP_SWEEP_M=$m python bench.py --workload doorkey65536 --method sweep --steps 3 --warmup 1 --no-cpu --no-hbm
done
echo all ok
