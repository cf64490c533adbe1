# The driver's bench command, REPS times (default 2): gpurun_out/$TAG/bench_<i>.{json,err}
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06_bench2}
mkdir -p $OUT
for i in $(seq 1 ${REPS:-2}); do
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { tail $OUT/bench_$i.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$OUT/bench_$i.json').read().strip().split(chr(10))[-1])
print(d['value'], d['ms_per_step'], {k: (v.get('v'), v.get('ms')) for k, v in d['configs'].items()})"
done
echo "all ok"
