# Config R (Empty-16 x 65536, the sweep method): the read+write copy ceiling on this box
# (tools/probe_copy) and the sweep kernel under its launch knobs (MGDP_SWEEP_PIPE depth,
# MGDP_SWEEP_GRID workgroups).  KNOBS "name=ENV=VAL,ENV=VAL ..." (default: a depth x grid sweep).
# Output: gpurun_out/$TAG/{copy.jsonl, sweep.jsonl, summary.txt}
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06_sweep}
mkdir -p $OUT
if [ -z "$SKIP_COPY" ]; then
  timeout -k 10 120 tools/probe_copy > $OUT/copy.jsonl 2> $OUT/copy.err || { cat $OUT/copy.err; echo "copy probe failed"; exit 1; }
  cat $OUT/copy.jsonl
fi
KNOBS=${KNOBS:-"base= p1=MGDP_SWEEP_PIPE=1 p3=MGDP_SWEEP_PIPE=3 p4=MGDP_SWEEP_PIPE=4 g1k=MGDP_SWEEP_GRID=1024 g4k=MGDP_SWEEP_GRID=4096 g8k=MGDP_SWEEP_GRID=8192 p3g4k=MGDP_SWEEP_PIPE=3,MGDP_SWEEP_GRID=4096"}
for rep in 1 2; do
  for spec in $KNOBS; do
    name=${spec%%=*}; envs=${spec#*=}
    timeout -k 10 300 env ${envs//,/ } python3 -u tools/probe_batch.py --method sweep --env MiniGrid-Empty-16x16-v0 --B 65536 \
      --solves 3 --reps 3 --tag $name >> $OUT/sweep.jsonl 2>> $OUT/sweep.err || { tail -20 $OUT/sweep.err; echo "sweep probe failed: $name"; exit 1; }
  done
done
python3 -c "
import json
for l in open('$OUT/sweep.jsonl'):
    d = json.loads(l)
    us = d['kernel_us'] * d['launches'] / (3 * d['sweeps'])  # speculative launches that exit at once included
    print('%-8s %8.2f us per sweep launch  %.3f TB/s compulsory (V in + out + cells)' % (d['tag'], us, (2 * 65536 * 4096 + 65536 * 256) / us / 1e6))
" | tee $OUT/summary.txt
echo "all ok"
