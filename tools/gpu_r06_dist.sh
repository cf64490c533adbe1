# Round 6: the sweep-chain probe (two sweeps per barrier variants 15 / 16) and the distributed GPU tests
# (mgdp_vi_solve_sharded at world 2 / 4 on one GPU through the host communicator; every mode vs the oracle).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06_dist}
mkdir -p $OUT
timeout -k 10 120 ./tools/probe_sweep_chain > $OUT/probe_sweep_chain.json 2>&1 || { cat $OUT/probe_sweep_chain.json; exit 1; }
cat $OUT/probe_sweep_chain.json
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_distributed.py > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
