# Cold-box lone-grid latency (TAG names the run; copy gpurun_out/$TAG to profiles/$TAG): the
# latency trajectory of the served Empty-16 solve from the first solve in a fresh lease
# (tools/probe_cold.py, trace build: per-1000-solve GPU-side time and s_memtime shader clock),
# then the driver's bench command with per-solve stamps, then the probe again on the product build.
# Needs exp_diag/trace/libmgdp.so:
#   MGDP_EXTRA_FLAGS=-DMGDP_SERVE_TRACE MGDP_BUILD_OUT=exp_diag/trace/libmgdp.so python -c "from minigrid_dynamicprogramming_amd import build; build.build()"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-cold}
mkdir -p $OUT
ls -l /sys/class/drm/card*/device/pp_dpm_sclk > $OUT/sysfs.txt 2>&1 || true
MGDP_LIB=exp_diag/trace/libmgdp.so timeout -k 10 120 python -u tools/probe_cold.py --out $OUT/cold_trace.json > $OUT/cold_trace.log 2> $OUT/cold_trace.err || { echo "probe failed"; tail -20 $OUT/cold_trace.err; exit 1; }
cat $OUT/cold_trace.log; grep "serve trace" $OUT/cold_trace.err | head -60
MGDP_BENCH_STAMPS=1 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench1.json 2> $OUT/bench1.err || { echo "bench failed"; tail $OUT/bench1.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench1.json')); print('bench', '%.4g'%d['value'], '%.3f us'%(d['ms_per_step']*1e3), 'f64 %.3f us'%(d['f64']['ms_per_step']*1e3))"
grep stamps $OUT/bench1.err
timeout -k 10 120 python -u tools/probe_cold.py --out $OUT/cold_prod.json > $OUT/cold_prod.log 2> $OUT/cold_prod.err || { echo "probe2 failed"; tail -20 $OUT/cold_prod.err; exit 1; }
cat $OUT/cold_prod.log
(timeout -k 5 60 amd-smi metric -g 0 --clock > $OUT/amdsmi_clock.txt 2>&1; true)
echo "all ok"
