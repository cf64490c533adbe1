# (Measured, not kept: U = 8 took 11.96 vs 10.45 us with U = 4; record of profiles/r02_reduce_u8/.)
# vi_reduce_kernel with 8 loads in flight per thread: parity of the large-batch paths, Lava x 65536
# bench and the reduce kernel's rocprofv3 duration.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02_reduce_u8
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_wave2.py tests/test_gpu_vi.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --workload lava65536 --steps 10 --warmup 2 --no-cpu --no-hbm --no-f64 > $OUT/rocprof_lava.json 2> $OUT/rocprof_lava.err || { echo "rocprof failed"; exit 1; }
python -c "import json; d=json.load(open('$OUT/rocprof_lava.json')); print('lava65536 (under rocprof)', '%.4g'%d['value'], '%.1f us/step'%(d['ms_per_step']*1e3))"
f=$(find $OUT/prof -name 'run_kernel_stats.csv' | head -1); grep -i "reduce" $f | cut -c1-170
echo "all ok"
