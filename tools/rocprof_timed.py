"""The timed launch in a rocprofv3 kernel trace of `bench.py`: the lone-grid server runs a warm
phase (its own launches, >= 200 ms) before the timed one, so the stats file's per-kernel average
mixes them; this prints each vi_serve_kernel dispatch and sets the last one (the timed launch, which
serves the relaunch-priming and the timed solves) beside the bench line's HIP-event launch time.

    python tools/rocprof_timed.py <run_kernel_trace.csv> <bench line .json> [out.json]"""
import csv
import json
import sys

trace, line = sys.argv[1], sys.argv[2]
rows = [r for r in csv.DictReader(open(trace)) if r["Kernel_Name"].startswith("void mgdp::vi_serve_kernel<float")]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
d = json.loads(open(line).read().strip().splitlines()[-1])
r = d["roofline"]
out = {
    "serve_dispatch_us": [round(x, 2) for x in durs],
    "timed_launch_us_rocprof": round(durs[-1], 2),
    "timed_launch_us_bench_events": round(r["avg_launch_us"], 2),
    "solves_per_launch": r["solves_per_launch"],
    "us_per_solve_rocprof": round(durs[-1] / r["solves_per_launch"], 3),
    "us_per_solve_bench_events": round(r["avg_launch_us"] / r["solves_per_launch"], 3),
    "note": "the earlier dispatches are the warm phase (bench.py two-phase priming, DESIGN 7); the last is the timed launch",
}
print(json.dumps(out, indent=1))
if len(sys.argv) > 3:
    json.dump(out, open(sys.argv[3], "w"), indent=1)
