"""Summarise rocprofv3 SQ counter passes for one kernel: per-dispatch means, the wave-cycle split
(WAIT_ANY / WAIT_INST_ANY / ACTIVE_INST_ANY, quad-cycles), VALU and LDS instructions per wave,
LDS-array busy fraction and the effective clock (GRBM_GUI_ACTIVE / 8 XCDs / kernel time)."""
import collections
import csv
import glob
import json
import sys

src, kernel = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "vi_fused_kernel")
agg = collections.defaultdict(list)
dur = []
for p in sorted(glob.glob(f"{src}_p*/run_counter_collection.csv")):
    seen = set()
    for r in csv.DictReader(open(p)):
        if r["Kernel_Name"].startswith(kernel):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Dispatch_Id"] not in seen:
                seen.add(r["Dispatch_Id"])
                dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
m = {k: sum(v) / len(v) for k, v in agg.items()}
t_us = sum(dur) / len(dur)
out = {"kernel": kernel, "avg_dispatch_us": t_us, "counters": m}
if "SQ_WAVE_CYCLES" in m:
    w = m["SQ_WAVE_CYCLES"]
    out["wave_split"] = {k: m[k] / w for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY") if k in m}
if "GRBM_GUI_ACTIVE" in m:
    cyc = m["GRBM_GUI_ACTIVE"] / 8
    out["clock_ghz"] = cyc / t_us / 1e3
    if "SQ_LDS_IDX_ACTIVE" in m:
        out["lds_array_busy"] = m["SQ_LDS_IDX_ACTIVE"] / 256 / cyc
    if "SQ_INSTS_VALU" in m:
        out["valu_instr_per_simd_cycle"] = m["SQ_INSTS_VALU"] / 1024 / cyc
if "SQ_WAVES" in m:
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
        if k in m:
            out[k + "_per_wave"] = m[k] / m["SQ_WAVES"]
print(json.dumps(out, indent=1))
