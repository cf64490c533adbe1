set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
timeout -k 10 300 python tools/probe_latency.py > gpurun_out/probe/latency_empty16.json 2>&1 && \
timeout -k 10 300 python tools/probe_latency.py MiniGrid-Empty-5x5-v0 > gpurun_out/probe/latency_empty5.json 2>&1
echo done $?
