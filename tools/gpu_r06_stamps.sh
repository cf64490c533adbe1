# Where the headline region's time goes (MGDP_BENCH_STAMPS: per-solve stamps, the closing
# synchronizes) and the batched blocks with the batch server relaunched before their regions.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06_stamps}
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 600 env MGDP_BENCH_STAMPS=1 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-hbm --no-f64 > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { tail $OUT/bench_$i.err; exit 1; }
  grep stamps_us $OUT/bench_$i.err | cut -c1-900
  tail -c 900 $OUT/bench_$i.json; echo
done
echo "all ok"
