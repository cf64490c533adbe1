# Quick perf probe: selected workloads, parity smoke first.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-quick}
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 600 python -m pytest tests/test_gpu_vi.py -x -q > $OUT/pytest_vi.log 2>&1 || { echo pytest failed; exit 1; }
run() { name=$1; shift; timeout -k 10 300 env "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; exit 1; }; }
run default python bench.py --no-cpu --no-hbm
for w in empty16x65536 lava65536 fourrooms4096 doorkey65536; do run ${w}_fused python bench.py --workload $w --steps 5 --warmup 1 --no-cpu --no-hbm; done
for b in 128 256; do for g in 2048 3072 4096 8192; do
  run R_sweep_b${b}_g${g} MGDP_SWEEP_BLOCK=$b MGDP_SWEEP_GRID=$g python bench.py --workload empty16x65536 --method sweep --steps 5 --warmup 1 --no-cpu --no-hbm
done; done
echo all ok
