# One-wave lone-grid path: VI parity tests, then default bench and per-sweep probes with the
# one-wave path on (MGDP_WAVE=8, default) and off (MGDP_WAVE=0, multi-wave loop).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-wave}
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests/test_gpu_vi.py -x -q > $OUT/pytest_vi.log 2>&1 || { echo pytest failed; tail -30 $OUT/pytest_vi.log; exit 1; }
for rep in 1 2; do
  for w in 8 0; do
    timeout -k 10 300 env MGDP_WAVE=$w python bench.py --no-cpu --no-hbm > $OUT/default_w${w}_r$rep.json 2> $OUT/default_w${w}_r$rep.err || { echo bench $w failed; exit 1; }
  done
done
for envid in MiniGrid-Empty-16x16-v0 MiniGrid-FourRooms-v0 MiniGrid-LavaCrossingS11N5-v0 MiniGrid-Empty-8x8-v0; do
  for w in 8 0; do
    timeout -k 10 300 env MGDP_WAVE=$w python tools/probe_sweep_cost.py $envid > $OUT/sweep_cost_${envid}_w$w.json 2>&1 || { echo probe $envid $w failed; exit 1; }
  done
done
echo all ok
