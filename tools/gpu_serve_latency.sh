# Lone-grid (served Empty-16x16) latency evidence (TAG names the run; copy gpurun_out/$TAG to
# profiles/$TAG): the served-path GPU tests, the LDS/barrier cost probe of one sweep, the NUMA
# probe, the C-ABI solve latency with and without fused_serve_xyd (MGDP_SERVE_EW) and vs the host's
# gap between solves with and without LDS-mailbox polling (MGDP_SERVE_POLL_DMA), the Python call
# overhead, and the driver's bench command (x2, 200 steps, and with MGDP_SERVE_EW=0).
# Needs the probes built in-tree (tools/README.md).
set -o pipefail
cd $GRAFT_REPO_ROOT
export OUT=gpurun_out/${TAG:-serve_latency}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_serve_ew.py tests/test_gpu_serve_grids.py tests/test_gpu_vi.py -m gpu > $OUT/pytest.log 2>&1 || { echo "tests failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 ./tools/probe_sweep_chain > $OUT/probe_sweep_chain.json 2>&1 || { echo "chain probe failed"; exit 1; }
timeout -k 10 200 ./tools/probe_numa > $OUT/numa.json 2>&1 || { echo "numa probe failed"; exit 1; }
for ew in 1 0; do
  MGDP_SERVE_EW=$ew timeout -k 10 120 ./tools/probe_serve ew$ew >> $OUT/serve.json 2>> $OUT/serve.err || { echo "probe failed"; exit 1; }
done
for dma in 1 0; do
  for g in 0 0.3 0.6 1 1.5 2 3; do
    MGDP_SERVE_POLL_DMA=$dma MGDP_PROBE_GAP_US=$g timeout -k 10 120 ./tools/probe_serve dma$dma >> $OUT/gap.json 2>> $OUT/gap.err || { echo "gap $g failed"; exit 1; }
  done
done
PYTHONPATH=. timeout -k 10 120 python tools/probe_solve_py.py > $OUT/py_solve.json 2> $OUT/py_solve.err || { echo "py probe failed"; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-hbm --no-sharded > $OUT/b$i.json 2> $OUT/b$i.err || { echo "bench failed"; tail $OUT/b$i.err; exit 1; }
done
timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 5 --no-cpu --no-hbm --no-sharded --no-f64 > $OUT/b200.json 2> $OUT/b200.err || exit 1
timeout -k 10 300 env MGDP_SERVE_EW=0 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-hbm --no-sharded > $OUT/b_ew0.json 2> $OUT/b_ew0.err || exit 1
grep '"max_sweeps": 10000' $OUT/serve.json
for f in $OUT/b*.json; do python -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', '%.4g'%d['value'], '%.3f us'%(d['ms_per_step']*1e3))"; done

# GPU-side request-seen -> publish time per solve (trace build in exp_diag/trace, if present):
# MGDP_EXTRA_FLAGS=-DMGDP_SERVE_TRACE MGDP_BUILD_OUT=exp_diag/trace/libmgdp.so python -c "from minigrid_dynamicprogramming_amd import build; build.build()"
if [ -f exp_diag/trace/libmgdp.so ]; then
  LD_LIBRARY_PATH=exp_diag/trace timeout -k 10 120 ./tools/probe_serve trace > $OUT/trace.json 2> $OUT/trace.err || { echo "trace probe failed"; exit 1; }
  grep "serve trace" $OUT/trace.err
fi
echo "all ok"
