# Round 5: is a batch that fills the one-wave kernel's resident capacity exactly (FourRooms x 4096 at
# 4 waves per SIMD, LavaS11N5 x 8192 at 8) dispatched in one round?  Kernel us per solve at B just
# under, at and just over the capacity (probe_batch -> cap.jsonl).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_cap}
mkdir -p $OUT
P="python3 -u tools/probe_batch.py --solves 10 --reps 3"
run() { timeout -k 10 150 env "$@" >> $OUT/cap.jsonl 2>> $OUT/cap.err || { echo "probe $* failed"; tail -5 $OUT/cap.err; exit 1; }; }
for B in 2048 3072 3584 3840 3968 4032 4096 4160 4608; do
  run MGDP_DEBUG_OCC=1 $P --tag fr --env MiniGrid-FourRooms-v0 --B $B || exit 1
done
for B in 4096 6144 7168 7680 7936 8128 8192 8256; do
  run $P --tag lava --env MiniGrid-LavaCrossingS11N5-v0 --B $B || exit 1
done
python3 -c "
import json
for l in open('$OUT/cap.jsonl'):
    d=json.loads(l); print('%-5s %-30s %6d %9.2f us %9.2f kern k %d x %.3f' % (d['tag'], d['env'], d['B'], d['us_per_solve'], d['kernel_us'], d['sweeps'], d['executed_frac']))"
grep -i occ $OUT/cap.err | sort | uniq -c | head
echo "all ok"
