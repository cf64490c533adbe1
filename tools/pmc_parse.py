"""Turn rocprofv3 --pmc passes (tools/pmc_traffic.sh) into profiles/pmc_traffic.json.

HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes).  The factor 2 is the gfx950
correction of MI355X_MICROARCH.md section HBM: FETCH_SIZE reports exactly half the bytes of a wide
coalesced streaming read.  Launches that wrote nothing (speculatively enqueued sweeps that exit
immediately) are excluded, matching bench.py's event accounting."""
import csv
import json
import os
import re
import sys
from collections import defaultdict

SRC = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
OUT = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_traffic.json"
# run -> (bench key, kernel, solves per launch for a persistent server launch or None); the grids one
# launch solves (bench.py scales traffic to a shard by it) is the number after the last "x" of the key
RUNS = {
    # --steps 20 --warmup 0: the timed launch serves the 16 priming solves and the 20 timed ones
    "empty16": ("empty16/fused/cell/f32", "vi_serve_kernel", 36),
    "empty16x65536_sweep": ("empty16x65536/sweep/cell/f32", "vi_sweep_pipe_kernel", None),
    "empty16x65536_fused": ("empty16x65536/fused/cell/f32", "vi_fused_kernel", None),
    "doorkey65536_fused": ("doorkey65536/fused/cell/f32", "vi_fused_kernel", None),
    "lava65536_fused": ("lava65536/fused/cell/f32", "vi_fused_kernel", None),
    "fourrooms4096_fused": ("fourrooms4096/fused/cell/f32", "vi_fused_kernel", None),
    # step / generator side benches (tools/pmc_side.sh); dword-wide scattered reads: the x2
    # correction is calibrated for 16-B streaming reads only (raw value kept beside it)
    "step_doorkey16x65536": ("step_doorkey16x65536/step", "envs_step_kernel", None),
    "step_fourrooms65536": ("step_fourrooms65536/step", "envs_step_kernel", None),
    "step_lava65536": ("step_lava65536/step", "envs_step_kernel", None),
    "step_doorkey16x1m": ("step_doorkey16x1m/step", "envs_step_kernel", None),
    "gen_lava65536": ("gen_lava65536/gen", "gen_grids_kernel", None),
    "gen_fourrooms65536": ("gen_fourrooms65536/gen", "gen_grids_kernel", None),
    "gen_doorkey16x65536": ("gen_doorkey16x65536/gen", "gen_grids_kernel", None),
}


def grids_of(key):
    """Grids (envs) one launch of the workload handles: the trailing count of its name ("lava65536",
    "empty16x65536", "step_doorkey16x1m"); a bare family name ("empty16") is the lone grid."""
    head = key.split("/")[0]
    m = re.search(r"x(\d+)(m?)$", head) or re.search(r"[a-z](\d{3,})(m?)$", head)
    if not m:
        return 1
    return int(m.group(1)) * ((1 << 20) if m.group(2) else 1)


def per_dispatch(path, kernel):
    vals = []
    for r in csv.DictReader(open(path)):
        if r["Kernel_Name"].startswith(kernel):
            vals.append(float(r["Counter_Value"]) * 1024.0)
    return vals


res = json.load(open(OUT)) if os.path.exists(OUT) else {}  # merge: passes come from several calls
for run, (key, kernel, solves) in RUNS.items():
    if not os.path.isdir(os.path.join(SRC, f"{run}_FETCH_SIZE")):
        continue
    f = per_dispatch(os.path.join(SRC, f"{run}_FETCH_SIZE", "run_counter_collection.csv"), kernel)
    w = per_dispatch(os.path.join(SRC, f"{run}_WRITE_SIZE", "run_counter_collection.csv"), kernel)
    n = min(len(f), len(w))
    # sweep method: drop the speculatively enqueued sweeps that exit at once (bench.py does not time
    # them); fused: every dispatch counts, as in bench.py's per-launch average (a chained solve's
    # run_to launch may have nothing to do)
    pairs = [(f[i], w[i]) for i in range(n) if w[i] > 4096 or "fused" in run or run == "empty16"]
    if solves:  # the timed server launch is the last one (warm-phase servers precede it)
        pairs = pairs[-1:]
    if not pairs:
        continue
    fetch = sum(p[0] for p in pairs) / len(pairs)
    write = sum(p[1] for p in pairs) / len(pairs)
    res[key] = {
        "kernel": kernel,
        "launches": len(pairs),
        "fetch_size_bytes_raw": fetch,
        "write_size_bytes": write,
        "bytes_per_launch": 2.0 * fetch + write,
        "note": "2*FETCH_SIZE + WRITE_SIZE per launch (gfx950 FETCH_SIZE half-count correction)",
    }
    if run.startswith(("step_", "gen_")):
        res[key]["note"] += "; dword/byte-wide accesses: the x2 is calibrated for 16-B streaming reads only"
    res[key]["src"] = SRC
    res[key]["grids_per_launch"] = grids_of(key)
    if solves:  # one resident launch served `solves` requests (bench.py scales per solve)
        res[key]["solves_per_launch"] = solves
        res[key]["bytes_per_solve"] = res[key]["bytes_per_launch"] / solves
os.makedirs(os.path.dirname(OUT), exist_ok=True)
json.dump(res, open(OUT, "w"), indent=1)
print(json.dumps(res, indent=1))
