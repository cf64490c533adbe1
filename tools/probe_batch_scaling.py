"""Per-launch time of the batched fused solve against the batch size (same family, seeds 0..B-1):
flat in B = latency-bound (the slowest grid's sweeps), linear = throughput-bound.  Prints one JSON
line per (env, B): solve wall time, launches per solve, average launch time, sweeps."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import minigrid_dynamicprogramming_amd as mg  # noqa: E402
from minigrid_dynamicprogramming_amd import gen  # noqa: E402

envs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["MiniGrid-FourRooms-v0"]
sizes = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [256, 1024, 2048, 4096, 8192, 16384]
for env_id in envs:
    for B in sizes:
        cells = gen.generate(env_id, 0, B, enc=False, cells=True, agent=False)["cells"]
        vi = mg.ValueIteration(cells, dtype=os.environ.get("DT", "f32"))
        for _ in range(3):
            vi.solve()
        vi.enable_timing(True)
        n = 10
        t0 = time.perf_counter()
        for _ in range(n):
            k = vi.solve()
        el = time.perf_counter() - t0
        ms, launches = vi.kernel_time()
        print(json.dumps({"env": env_id, "B": B, "sweeps": k, "us_per_solve": el / n * 1e6,
                          "launches_per_solve": launches / n, "us_per_launch": ms * 1e3 / max(launches, 1),
                          "updates_per_s": B * vi.S * 7 * k / (el / n)}), flush=True)
        vi.close()
