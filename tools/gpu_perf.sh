# Perf pass: VI parity tests, then the default bench and every workload (fused), R sweep.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-perf}
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_gpu_vi.py -x -q > $OUT/pytest_vi.log 2>&1 || { echo pytest failed; exit 1; }
run() { name=$1; shift; timeout -k 10 300 env "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "$name failed"; exit 1; }; }
run default python bench.py --no-cpu --no-hbm
for w in empty16x65536 lava65536 fourrooms4096 doorkey65536; do run ${w}_fused python bench.py --workload $w --steps 5 --warmup 1 --no-cpu --no-hbm; done
run empty16x65536_sweep python bench.py --workload empty16x65536 --method sweep --steps 5 --warmup 1 --no-cpu --no-hbm
run doorkey65536_sweep python bench.py --workload doorkey65536 --method sweep --steps 2 --warmup 1 --no-cpu --no-hbm
echo all ok
