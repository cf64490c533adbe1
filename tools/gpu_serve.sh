# Persistent-server check: VI parity tests, smoke, default bench with and without the server.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-serve}
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests/test_gpu_vi.py -x -q > $OUT/pytest_vi.log 2>&1 || { echo pytest failed; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; exit 1; }
timeout -k 10 300 python bench.py --no-cpu --no-hbm > $OUT/default.json 2> $OUT/default.err || { echo bench failed; exit 1; }
timeout -k 10 300 env MGDP_PERSISTENT=0 python bench.py --no-cpu --no-hbm > $OUT/default_nopersist.json 2> $OUT/default_nopersist.err || { echo bench0 failed; exit 1; }
timeout -k 10 300 python tools/probe_latency.py > $OUT/latency_empty16.json 2>&1 || { echo probe failed; exit 1; }
timeout -k 10 300 python tools/probe_sweep_cost.py > $OUT/sweep_cost.json 2>&1 || { echo probe2 failed; exit 1; }
timeout -k 10 300 env MGDP_PAIR=1 python tools/probe_sweep_cost.py > $OUT/sweep_cost_pair.json 2>&1 || { echo probe4 failed; exit 1; }
timeout -k 10 300 env MGDP_PAIR=1 python bench.py --no-cpu --no-hbm > $OUT/default_pair.json 2> $OUT/default_pair.err || { echo bench_pair failed; exit 1; }
echo all ok
