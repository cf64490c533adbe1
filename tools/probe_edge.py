"""The timed region's closing edge for the served lone grid: after the last solve (solve_last), how
long mgdp_vi_synchronize (the server's exit word) and torch.cuda.synchronize (the stream's
completion) take, against how long the server ran before (priming length) and whether launch
timing (HIP events around the server launch) is on.  One JSON line per configuration (medians of
--reps runs)."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--prime-ms", default="0.1,2,20,200")
    args = ap.parse_args()
    import torch

    import minigrid_dynamicprogramming_amd as mg
    from minigrid_dynamicprogramming_amd import _lib

    _lib.pin_host_thread(0)
    enc, _ = mg.make("MiniGrid-Empty-16x16-v0").generate(seed=0)
    vi = mg.ValueIteration(np.ascontiguousarray(enc[..., 0].T)[None], dtype="f32")
    torch.cuda.synchronize()
    for timing in (True, False):
        for pm in [float(x) for x in args.prime_ms.split(",")]:
            rows = []
            for _ in range(args.reps):
                vi.enable_timing(timing)
                torch.cuda.synchronize()
                t_end = time.perf_counter() + pm / 1e3
                n = 0
                while True:
                    vi.solve()
                    n += 1
                    if time.perf_counter() >= t_end:
                        break
                t0 = time.perf_counter()
                for i in range(20):
                    vi.solve(last=i == 19)
                t1 = time.perf_counter()
                vi.synchronize()
                t2 = time.perf_counter()
                torch.cuda.synchronize()
                t3 = time.perf_counter()
                rows.append(((t1 - t0) * 1e6 / 20, (t2 - t1) * 1e6, (t3 - t2) * 1e6, n))
            r = np.array(rows)
            print(json.dumps({"timing": timing, "prime_ms": pm, "primed_solves": int(np.median(r[:, 3])),
                              "solve_us": round(float(np.median(r[:, 0])), 3),
                              "vi_sync_us": round(float(np.median(r[:, 1])), 2),
                              "dev_sync_us": round(float(np.median(r[:, 2])), 2),
                              "dev_sync_all": [round(x, 1) for x in r[:, 2]]}), flush=True)
    vi.close()


if __name__ == "__main__":
    main()
