set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02f
mkdir -p $OUT
MGDP_BENCH_STAMPS=1 timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-hbm > $OUT/bench_s20.json 2> $OUT/bench_s20.err || { echo "bench failed"; tail $OUT/bench_s20.err; exit 1; }
grep stamps $OUT/bench_s20.err
