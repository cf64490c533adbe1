# Register-pipelined HBM sweep kernel: VI parity tests, then sweep-method benches per depth
# (MGDP_SWEEP_PIPE=0 staged kernel, 1, 2).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pipe}
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests/test_gpu_vi.py tests/test_gpu_distributed.py -x -q > $OUT/pytest_vi.log 2>&1 || { echo pytest failed; tail -30 $OUT/pytest_vi.log; exit 1; }
for w in empty16x65536 lava65536 fourrooms4096 doorkey65536; do
  for p in 0 1 2; do
    timeout -k 10 300 env MGDP_SWEEP_PIPE=$p python bench.py --workload $w --method sweep --steps 3 --warmup 1 --no-cpu --no-hbm > $OUT/${w}_p$p.json 2> $OUT/${w}_p$p.err || { echo "$w $p failed"; exit 1; }
  done
done
echo all ok
