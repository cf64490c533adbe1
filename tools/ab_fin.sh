mkdir -p gpurun_out/r04_finab
for rep in 1 2; do
for lib in minigrid_dynamicprogramming_amd/libmgdp.so abl/fin/libmgdp.so; do
for w in "MiniGrid-LavaCrossingS11N5-v0 65536" "MiniGrid-FourRooms-v0 4096" "MiniGrid-Empty-16x16-v0 65536"; do
set -- $w
MGDP_LIB=$lib timeout -k 10 100 python -u tools/probe_batch.py --env $1 --B $2 --tag "$lib" >> gpurun_out/r04_finab/ab.jsonl 2>> gpurun_out/r04_finab/ab.err || exit 1
done; done; done
python -c "
import json
for l in open('gpurun_out/r04_finab/ab.jsonl'):
    d=json.loads(l); print(d['tag'][:30], d['env'][9:20], d['B'], d['us_per_solve'], d['kernel_us'], '%.3g'%d['updates_per_s'])"
