# Round 5: A/B of the tree build against ablib/libmgdp_nopf.so -- first fused_wave2_xyd reading the next sweep's fronts right after its stores (MGDP_WAVE2_PREFETCH=1,
# the tree's build) vs each sweep reading its own (ablib/libmgdp_nopf.so, MGDP_LIB): the wave2 GPU
# tests, then probe_batch A/B -> ab.jsonl.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_pf}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wave2.py tests/test_gpu_fixedpoint.py tests/test_gpu_fullsize.py tests/test_gpu_mix.py -k "not capacity" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; echo "tests failed"; exit 1; }
tail -1 $OUT/pytest.log
P="python3 -u tools/probe_batch.py --solves 10 --reps 3"
run() { tag=$1; shift; kv=(); while [[ "$1" == *=* ]]; do kv+=("$1"); shift; done; timeout -k 10 150 env "${kv[@]}" $P --tag $tag "$@" >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "probe $tag failed"; tail -5 $OUT/ab.err; exit 1; }; }
for rep in 1 2; do
  for wl in "MiniGrid-LavaCrossingS11N5-v0 65536" "MiniGrid-LavaCrossingS11N5-v0 8192" "MiniGrid-FourRooms-v0 4096" "MiniGrid-Empty-16x16-v0 65536"; do set -- $wl
    run ${BASE_LABEL:-nopf} MGDP_LIB=ablib/libmgdp_nopf.so --env $1 --B $2 || exit 1
    run ${NEW_LABEL:-pf} MGDP_NOP=1 --env $1 --B $2 || exit 1
  done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print('%-6s %-30s %6d %9.2f us %9.2f kern %.4g upd/s' % (d['tag'], d['env'], d['B'], d['us_per_solve'], d['kernel_us'], d['updates_per_s']))"
echo "all ok"
