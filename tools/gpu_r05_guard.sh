# Round 5: host path of a batched solve -- one device guard per mgdp_vi_solve (nested guards make no
# runtime call) and the occupancy-diagnostics getenv read once -- vs the build before
# (ablib/libmgdp_base.so, MGDP_LIB): the full GPU suite, then probe_batch wall / kernel A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_guard}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; echo "tests failed"; exit 1; }
tail -1 $OUT/pytest.log
P="python3 -u tools/probe_batch.py --solves 20 --reps 5"
for rep in 1 2 3; do
  for wl in "MiniGrid-LavaCrossingS11N5-v0 8192" "MiniGrid-LavaCrossingS11N5-v0 512" "MiniGrid-FourRooms-v0 4096"; do set -- $wl
    for lib in base new; do
      L=""; [ $lib = base ] && L=ablib/libmgdp_base.so
      timeout -k 10 150 env MGDP_LIB=$L $P --tag $lib --env $1 --B $2 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "probe failed"; exit 1; }
    done
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print('%-4s %-30s %6d %9.2f us %9.2f kern %.4g upd/s' % (d['tag'], d['env'], d['B'], d['us_per_solve'], d['kernel_us'], d['updates_per_s']))"
echo "all ok"
