# Round 5: per-sweep cost and fixed work of the batched one-wave kernel by occupancy (max_sweeps
# caps, tools/probe_batch_caps.py): FourRooms (P = 6) and LavaS11N5 (P = 2) at 1..8 waves per SIMD.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_caps}
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/probe_batch_caps.py --env MiniGrid-FourRooms-v0 --B 256 1024 2048 4096 > $OUT/caps.jsonl 2> $OUT/caps.err || { tail $OUT/caps.err; exit 1; }
timeout -k 10 300 python3 -u tools/probe_batch_caps.py --env MiniGrid-LavaCrossingS11N5-v0 --B 256 1024 4096 8192 --caps 1 2 4 8 16 32 0 >> $OUT/caps.jsonl 2>> $OUT/caps.err || { tail $OUT/caps.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/caps.jsonl'):
    d=json.loads(l); print(d['env'][9:20], d['B'], ' '.join('%s:%s/%.1f' % (c, v['k'], v['kernel_us']) for c, v in d['caps'].items()))"
echo "all ok"
