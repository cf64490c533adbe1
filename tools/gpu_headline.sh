set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/head1
mkdir -p $OUT
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo bench failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d $OUT/prof_default -o run --output-format csv -- python3 bench.py --warmup 0 --no-cpu --no-hbm > $OUT/prof_default.log 2>&1 || { echo rocprof failed; exit 1; }
echo ok
