set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dist
timeout -k 10 600 python -m pytest tests/test_gpu_distributed.py -x -q > gpurun_out/dist/pytest.log 2>&1 || { echo pytest failed; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 2 > gpurun_out/dist/torchrun_default.json 2> gpurun_out/dist/torchrun_default.err || { echo torchrun default failed; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --workload lava65536 --steps 3 --warmup 1 > gpurun_out/dist/torchrun_lava.json 2> gpurun_out/dist/torchrun_lava.err || { echo torchrun lava failed; exit 1; }
echo dist ok
