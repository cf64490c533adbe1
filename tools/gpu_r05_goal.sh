# Round 5: DoorKey rows with the goal reward as one select (KD waves: no walkability mask) vs the
# build before (ablib/libmgdp_base.so, MGDP_LIB): the DoorKey GPU tests, then probe_batch A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_goal}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dk_rows.py tests/test_gpu_fullsize.py tests/test_gpu_fixedpoint.py $(ls tests/test_gpu_dk*.py | grep -v dk_rows) -k "not capacity" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; echo "tests failed"; exit 1; }
tail -1 $OUT/pytest.log
P="python3 -u tools/probe_batch.py --solves 5 --reps 3"
for rep in 1 2; do
  for lib in base new; do
    L=""; [ $lib = base ] && L=ablib/libmgdp_base.so
    timeout -k 10 200 env MGDP_LIB=$L $P --tag $lib --env MiniGrid-DoorKey-16x16-v0 --B 65536 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "probe failed"; exit 1; }
    timeout -k 10 200 env MGDP_LIB=$L $P --tag $lib --env MiniGrid-DoorKey-16x16-v0 --B 8192 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "probe failed"; exit 1; }
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print('%-4s %6d %9.2f us %9.2f kern %.4g upd/s' % (d['tag'], d['B'], d['us_per_solve'], d['kernel_us'], d['updates_per_s']))"
echo "all ok"
