# Quick iteration pass: a pytest selection (K=expr) and a few bench workloads (WL="a b c").
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-iter}
mkdir -p $OUT
if [ -n "$K" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
fi
for w in $WL; do
timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-10} --warmup 2 --no-cpu --no-hbm --no-f64 $BARGS > $OUT/bench_$w.json 2> $OUT/bench_$w.err || { echo "bench $w failed"; tail $OUT/bench_$w.err; exit 1; }
python -c "import json,sys; d=json.load(open('$OUT/bench_$w.json')); print('$w', '%.4g'%d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_us'])"
done
echo "all ok"
