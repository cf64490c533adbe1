# Round 5: the in-launch reduction's last level folded by the host (MGDP_GK_HOSTFOLD=1, default: each
# shard's last grid publishes three epoch-tagged words) vs in the launch (=0): the full GPU suite,
# then probe_batch A/B on the resident batches -> ab.jsonl.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_hostfold}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; echo "tests failed"; exit 1; }
tail -1 $OUT/pytest.log
P="python3 -u tools/probe_batch.py --solves 10 --reps 3"
for rep in 1 2; do
  for wl in "MiniGrid-LavaCrossingS11N5-v0 8192" "MiniGrid-FourRooms-v0 4096" "MiniGrid-Empty-16x16-v0 4096" "MiniGrid-LavaCrossingS11N5-v0 512"; do set -- $wl
    for hf in 0 1; do
      timeout -k 10 150 env MGDP_GK_HOSTFOLD=$hf $P --tag hf$hf --env $1 --B $2 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "probe failed"; exit 1; }
    done
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print('%-4s %-30s %6d %9.2f us %9.2f kern %.4g upd/s' % (d['tag'], d['env'], d['B'], d['us_per_solve'], d['kernel_us'], d['updates_per_s']))"
echo "all ok"
