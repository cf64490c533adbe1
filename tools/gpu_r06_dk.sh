set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06_dk
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dk_rows.py tests/test_gpu_fullsize.py > gpurun_out/r06_dk/pytest.log 2>&1 || { tail -30 gpurun_out/r06_dk/pytest.log; exit 1; }
tail -2 gpurun_out/r06_dk/pytest.log
TAG=r06_dk LIBS="r05=$PWD/ablib/libmgdp_r05.so new=" CONFIGS="MiniGrid-DoorKey-16x16-v0:65536 MiniGrid-DoorKey-16x16-v0:8192" REPS=2 bash tools/gpu_ab_batch.sh
