# (Measured, not kept: 20 ms of priming measured the same as 16 solves; record of profiles/r02_prime/.)
# Default bench (the driver's command) three times in fresh processes, 20 ms priming (default) vs
# the old 16 solves (MGDP_BENCH_PRIME_MS=0), first-process effect included.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02_prime
mkdir -p $OUT
for i in 1 2 3; do
for pm in 20 0; do
MGDP_BENCH_PRIME_MS=$pm timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-hbm > $OUT/p${pm}_$i.json 2> $OUT/p${pm}_$i.err || { echo "bench failed"; tail $OUT/p${pm}_$i.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/p${pm}_$i.json')); print('prime_ms $pm run $i', '%.4g'%d['value'], '%.3f us'%(d['ms_per_step']*1e3), 'f64 %.4g'%d['f64']['value'], 'primed', d['roofline']['solves_per_launch']-20)"
done
done
echo "all ok"
