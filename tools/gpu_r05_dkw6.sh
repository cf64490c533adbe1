# Round 5: fused_dk_rows compiled for 6 waves per SIMD (MGDP_DKROW_MINW=6: 80 VGPRs + 80 B of
# scratch, 6 grids per CU) vs the default 5 (100 VGPRs): the DoorKey rows tests on the 6-wave build
# (MGDP_LIB), then probe_batch A/B -> ab.jsonl.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_dkw6}
mkdir -p $OUT
MGDP_LIB=ablib/libmgdp_dkw6.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dk_rows.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; echo "tests failed"; exit 1; }
tail -1 $OUT/pytest.log
P="python3 -u tools/probe_batch.py --solves 5 --reps 3"
for rep in 1 2; do
  for lib in w5 w6; do
    L=""; [ $lib = w6 ] && L=ablib/libmgdp_dkw6.so
    timeout -k 10 200 env MGDP_LIB=$L $P --tag $lib --env MiniGrid-DoorKey-16x16-v0 --B 65536 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "probe failed"; exit 1; }
    timeout -k 10 200 env MGDP_LIB=$L $P --tag $lib --env MiniGrid-DoorKey-16x16-v0 --B 8192 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "probe failed"; exit 1; }
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print('%-4s %6d %9.2f us %9.2f kern %.4g upd/s' % (d['tag'], d['B'], d['us_per_solve'], d['kernel_us'], d['updates_per_s']))"
echo "all ok"
