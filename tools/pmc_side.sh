# PMC HBM traffic of the step and generator kernels (FETCH_SIZE / WRITE_SIZE in separate passes,
# kernel trace only), parsed by tools/pmc_parse.py into profiles/pmc_traffic.json.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc}
mkdir -p $OUT
prof() { name=$1; ctr=$2; shift 2
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace -T -d $OUT/${name}_${ctr} -o run --output-format csv -- python3 bench.py "$@" --no-cpu > $OUT/${name}_${ctr}.log 2>&1 || { echo "$name $ctr failed"; exit 1; }; }
for c in FETCH_SIZE WRITE_SIZE; do
  prof step_doorkey16x65536 $c --workload step_doorkey16x65536 --steps 5 --warmup 1
  prof step_fourrooms65536 $c --workload step_fourrooms65536 --steps 5 --warmup 1
  prof step_lava65536 $c --workload step_lava65536 --steps 5 --warmup 1
  prof gen_lava65536 $c --workload gen_lava65536 --steps 3 --warmup 1
  prof gen_fourrooms65536 $c --workload gen_fourrooms65536 --steps 3 --warmup 1
  prof gen_doorkey16x65536 $c --workload gen_doorkey16x65536 --steps 3 --warmup 1
done
echo pmc ok
