# A/B: vi_sweep_kernel (DoorKey sweep method) with nontemporal V copies vs the previous build.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/nt2; mkdir -p $OUT
L=minigrid_dynamicprogramming_amd/libmgdp.so
cp $L gpurun_out/libmgdp_new.so
run() { timeout -k 10 300 python bench.py --workload doorkey65536 --method sweep --steps 3 --warmup 1 --no-cpu >> $OUT/$1.jsonl 2>> $OUT/err || exit 1; }
for i in 1 2; do
  cp tools/exp/libmgdp_prev.so $L && run prev
  cp gpurun_out/libmgdp_new.so $L && run new
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_vi.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_vi.log 2>&1 || exit 1
rm gpurun_out/libmgdp_new.so
echo ok
