# Round 5: two waves per grid (fused_wave2n_xyd, MGDP_WAVE2N=1) after its loop got the stop test at
# the end of the deciding sweep, at the compiler's 6 waves per SIMD (80 VGPRs) and built for 8
# (ablib/libmgdp_w2n8.so: 64 VGPRs + 56 B scratch), against one wave per grid (fused_wave2_xyd):
# the two-wave tests on both builds, then probe_batch A/B -> ab.jsonl.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_w2n}
mkdir -p $OUT
for L in "" ablib/libmgdp_w2n8.so; do
  MGDP_LIB=$L timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread $(grep -ln MGDP_WAVE2N tests/*.py) tests/test_gpu_mix.py > $OUT/pytest$(basename "$L").log 2>&1 || { tail -40 $OUT/pytest$(basename "$L").log; echo "tests failed"; exit 1; }
  tail -1 $OUT/pytest$(basename "$L").log
done
P="python3 -u tools/probe_batch.py --solves 10 --reps 3"
run() { tag=$1; shift; kv=(); while [[ "$1" == *=* ]]; do kv+=("$1"); shift; done; timeout -k 10 150 env "${kv[@]}" $P --tag $tag "$@" >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "probe $tag failed"; tail -5 $OUT/ab.err; exit 1; }; }
for rep in 1 2; do
  for wl in "MiniGrid-FourRooms-v0 4096" "MiniGrid-FourRooms-v0 2048" "MiniGrid-Empty-16x16-v0 4096"; do set -- $wl
    run wave2 MGDP_WAVE2N=0 --env $1 --B $2 || exit 1
    run w2n_w6 MGDP_WAVE2N=1 --env $1 --B $2 || exit 1
    run w2n_w8 MGDP_WAVE2N=1 MGDP_LIB=ablib/libmgdp_w2n8.so --env $1 --B $2 || exit 1
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print('%-7s %-26s %6d %9.2f us %9.2f kern %.4g upd/s' % (d['tag'], d['env'], d['B'], d['us_per_solve'], d['kernel_us'], d['updates_per_s']))"
echo "all ok"
