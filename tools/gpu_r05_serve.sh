# Round 5: the served lone grid on one column-band wave (MGDP_SERVE_BAND=1, fused_band_xyd) vs the
# 4-wave fused_serve_xyd server: served-path GPU tests with the band server, then the headline bench
# (no blocks, no CPU legs) alternating the two, REPS times, STEPS timed solves each.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r05_serve}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_band.py ${EXTRA_TESTS:-} -k "not capacity" > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
MGDP_SERVE_BAND=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_serve_grids.py tests/test_gpu_resume.py -m gpu > $OUT/pytest_served.log 2>&1 || { echo "served tests failed"; tail -30 $OUT/pytest_served.log; exit 1; }
tail -1 $OUT/pytest_served.log
for rep in $(seq ${REPS:-3}); do
  for sb in 1 0; do
    n=band${sb}_$rep
    MGDP_SERVE_BAND=$sb timeout -k 10 200 python bench.py --gpus 1 --steps ${STEPS:-200} --warmup 5 --no-cpu --no-hbm --no-sharded --no-f64 > $OUT/$n.json 2> $OUT/$n.err || { echo "bench $n failed"; tail $OUT/$n.err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); l=d.get('lat_us',{}); print('$n', '%.4g'%d['value'], '%.3f us'%(d['ms_per_step']*1e3), 'gpu', l.get('gpu'), 'host', l.get('host'), 'sweeps', d['sweeps'])"
  done
done
for kn in "MGDP_LEARN_ORDER=1" "MGDP_LEARN_ORDER=0" "MGDP_LEARN_ORDER=1 MGDP_LEARN_PRIO=1"; do
  timeout -k 10 200 python tools/probe_capacity.py $kn >> $OUT/capacity.jsonl 2>> $OUT/capacity.err || { echo "capacity probe failed"; tail $OUT/capacity.err; exit 1; }
done
cat $OUT/capacity.jsonl
echo all ok
