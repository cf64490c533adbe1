# Round 5: the epoch-tagged host publication (four tagged words, no drain between them) against the
# build before it (ablib/libmgdp_r05pre.so, MGDP_LIB): rank 0's 8-way LavaS11N5 / DoorKey-16 shard,
# direct and through the library communicator, timed without per-launch events in the region
# (MGDP_BENCH_SPLIT_EVENTS=1, as the default line's blocks run), plus probe_batch wall vs kernel time.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_proto}
mkdir -p $OUT
summ() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('%-28s'%'$2', d['config']['grids_per_gpu'], 'grids', '%.4g'%d['value'], '%.2f us/solve'%(d['ms_per_step']*1e3), '%.2f us/launch'%r['avg_launch_us'], d.get('collectives',{}).get('path'))"; }
for rep in 1 2; do
for lib in pre cur; do
  L=""; [ $lib = pre ] && L=ablib/libmgdp_r05pre.so
  for w in lava65536 doorkey65536; do
    timeout -k 10 300 env MGDP_LIB=$L MGDP_BENCH_SPLIT_EVENTS=1 MGDP_BENCH_SHARD_OF=8 python bench.py --workload $w --steps 40 --warmup 5 --no-cpu --no-hbm --no-f64 > $OUT/direct_${lib}_${w}_$rep.json 2> $OUT/direct_${lib}_${w}_$rep.err || { echo "direct $lib $w failed"; tail $OUT/direct_${lib}_${w}_$rep.err; exit 1; }
    summ $OUT/direct_${lib}_${w}_$rep.json direct_${lib}_${w}_$rep
    timeout -k 10 300 env MGDP_LIB=$L MGDP_BENCH_SPLIT_EVENTS=1 MGDP_BENCH_SHARD_OF=8 MGDP_BENCH_FORCE_DIST=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29000 + RANDOM % 1000)) \
      bench.py --workload $w --steps 40 --warmup 5 --no-cpu --no-hbm --no-f64 > $OUT/lib_${lib}_${w}_$rep.json 2> $OUT/lib_${lib}_${w}_$rep.err || { echo "lib $lib $w failed"; tail $OUT/lib_${lib}_${w}_$rep.err; exit 1; }
    summ $OUT/lib_${lib}_${w}_$rep.json lib_${lib}_${w}_$rep
  done
  for wl in "MiniGrid-FourRooms-v0 4096" "MiniGrid-LavaCrossingS11N5-v0 8192" "MiniGrid-LavaCrossingS11N5-v0 512"; do set -- $wl
    timeout -k 10 150 env MGDP_LIB=$L python3 -u tools/probe_batch.py --solves 10 --reps 3 --tag $lib --env $1 --B $2 >> $OUT/ab.jsonl 2>> $OUT/ab.err || { echo "probe failed"; exit 1; }
  done
done
done
python3 -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print('%-6s %-30s %6d %9.2f us %9.2f kern gap %.2f' % (d['tag'], d['env'], d['B'], d['us_per_solve'], d['kernel_us'], d['us_per_solve'] - d['kernel_us']))"
echo "all ok"
