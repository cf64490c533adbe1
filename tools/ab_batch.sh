# A/B of batched solves across builds: ALT names the alternative library (an MGDP_BUILD_OUT build),
# ENVS the "env_id B" pairs, TAG the run; REPS alternations of tools/probe_batch.py per pair.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-ab_batch}
mkdir -p $OUT
for rep in $(seq ${REPS:-2}); do
  for lib in minigrid_dynamicprogramming_amd/libmgdp.so $ALT; do
    echo "${ENVS:-MiniGrid-DoorKey-16x16-v0 65536}" | tr ';' '\n' | while read env B; do
      MGDP_LIB=$lib timeout -k 10 120 python -u tools/probe_batch.py --env $env --B $B --solves ${SOLVES:-10} --reps 3 --tag "$lib" >> $OUT/ab.jsonl 2>> $OUT/ab.err || exit 1
    done || exit 1
  done
done
python -c "
import json
for l in open('$OUT/ab.jsonl'):
    d=json.loads(l); print(d['tag'][:40], d['env'][9:22], d['B'], d['us_per_solve'], d['kernel_us'], '%.4g'%d['updates_per_s'], d['sweeps'], d['executed_frac'])"
echo all ok
