# A/B: vi_sweep_pipe_kernel with nontemporal V stores (nt1) and stores+loads (nt3) vs the default build.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/nt; mkdir -p $OUT
L=minigrid_dynamicprogramming_amd/libmgdp.so
cp $L $OUT/../libmgdp_base.so
run() { timeout -k 10 300 python bench.py --workload empty16x65536 --method sweep --steps 5 --warmup 1 --no-cpu >> $OUT/$1.jsonl 2>> $OUT/err || exit 1; }
for i in 1 2; do
  cp gpurun_out/libmgdp_base.so $L && run base
  cp tools/exp/libmgdp_nt1.so $L && run nt1
  cp tools/exp/libmgdp_nt3.so $L && run nt3
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_vi.py -m gpu -x -q -k "sweep or pipe" --timeout 120 --timeout-method thread > $OUT/pytest_nt3.log 2>&1 || exit 1
rm gpurun_out/libmgdp_base.so
echo ok
