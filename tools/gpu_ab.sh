# A/B of two library builds on the same box: default libmgdp.so vs $B_LIB (e.g. exp/libmgdp_nopk.so),
# alternating twice, on workloads $WL.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
for rep in 1 2; do
for lib in minigrid_dynamicprogramming_amd/libmgdp.so $B_LIB; do
for w in ${WL:-empty16x65536 lava65536 fourrooms4096}; do
n=$(basename $lib .so)
MGDP_LIB=$PWD/$lib timeout -k 10 120 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu --no-hbm --no-f64 > $OUT/${n}_${w}_$rep.json 2> $OUT/${n}_${w}_$rep.err || { echo "$lib $w failed"; tail $OUT/${n}_${w}_$rep.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/${n}_${w}_$rep.json')); print('$n $w', '%.4g'%d['value'], '%.1f'%d['roofline']['avg_launch_us'])"
done
done
done
