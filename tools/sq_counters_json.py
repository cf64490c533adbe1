"""profiles/sq_counters.json from the SQ counter summaries (tools/sq_summary.py output) that
bench.py's roofline blocks read: per-launch VALU / LDS wave-instructions, VALU issue fraction
(a wave64 VALU instruction issues over 2 cycles: peak 0.5 per SIMD-cycle, MI355X_MICROARCH.md),
LDS-array busy fraction, wave-cycle split.  Usage: python tools/sq_counters_json.py KEY=SUMMARY..."""
import json
import os
import re
import sys

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "sq_counters.json")
res = json.load(open(OUT)) if os.path.exists(OUT) else {}
for arg in sys.argv[1:]:
    key, path = arg.split("=", 1)
    s = json.load(open(path))
    c = s["counters"]
    res[key] = {
        "valu_insts_per_launch": c["SQ_INSTS_VALU"],
        "lds_insts_per_launch": c.get("SQ_INSTS_LDS"),
        "waves_per_launch": c.get("SQ_WAVES"),
        "valu_issue_frac": s["valu_instr_per_simd_cycle"] / 0.5,
        "lds_array_busy": s.get("lds_array_busy"),
        "wave_split": s.get("wave_split"),
        "avg_dispatch_us_under_pmc": s["avg_dispatch_us"],
        # the grids one launch solved (bench.py scales per-launch counts to a shard by it)
        "grids_per_launch": int(re.search(r"(\d+)/", key).group(1)),
        "source": os.path.relpath(path, os.path.dirname(os.path.dirname(OUT))),
    }
json.dump(res, open(OUT, "w"), indent=1)
print(json.dumps(res, indent=1))
