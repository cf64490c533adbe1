# Round 5: what the in-launch reduction tree costs a resident launch: kernel us per solve (all
# launches of the solve) under max_sweeps caps with the tree (MGDP_GK=2, default) and with the
# reduce kernel instead (MGDP_GK=0), FourRooms and LavaS11N5 at one and at full residency.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_gkcost}
mkdir -p $OUT
for gk in 2 0; do
  timeout -k 10 200 env MGDP_GK=$gk python3 -u tools/probe_batch_caps.py --env MiniGrid-FourRooms-v0 --B 256 4096 --caps 1 8 0 > $OUT/caps_gk$gk.jsonl 2>> $OUT/caps.err || { echo "caps failed"; exit 1; }
  timeout -k 10 200 env MGDP_GK=$gk python3 -u tools/probe_batch_caps.py --env MiniGrid-LavaCrossingS11N5-v0 --B 256 8192 --caps 1 8 0 >> $OUT/caps_gk$gk.jsonl 2>> $OUT/caps.err || { echo "caps failed"; exit 1; }
  python3 -c "
import json
for l in open('$OUT/caps_gk$gk.jsonl'):
    d=json.loads(l); print('gk$gk', d['env'][9:20], d['B'], ' '.join('%s:%s/%.1f(%d)' % (c, v['k'], v['kernel_us_per_solve'], v['launches']) for c, v in d['caps'].items()))"
done
echo "all ok"
