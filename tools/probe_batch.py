"""One batched solve configuration, timed: wall per solve with launch timing off, kernel time per
solve with it on (HIP events), sweeps and the executed fraction.  For A/B runs across builds
(MGDP_LIB) and knobs (MGDP_* env).  Prints one JSON line."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="MiniGrid-FourRooms-v0")
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--solves", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--tag", default="")
    ap.add_argument("--method", default="fused")
    args = ap.parse_args()
    import torch

    import minigrid_dynamicprogramming_amd as mg
    from minigrid_dynamicprogramming_amd import _lib, gen

    _lib.pin_host_thread(0)
    cells = gen.generate(args.env, 0, args.B, enc=False, cells=True, agent=False)["cells"]
    vi = mg.ValueIteration(cells, dtype=args.dtype, method=args.method)
    wall, kern = [], []
    for _ in range(args.reps):
        vi.enable_timing(False)
        vi.solve()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.solves):
            k = vi.solve()
        wall.append((time.perf_counter() - t) * 1e6 / args.solves)
        vi.enable_timing(True)
        for _ in range(args.solves):
            vi.solve()
        ms, n = vi.kernel_time()
        kern.append(ms * 1e3 / max(n, 1))  # per launch (the sweep method: one launch per sweep)
        launches = n
    gs = vi.grid_sweeps()
    upd = vi.updates_per_sweep * k
    print(json.dumps({"tag": args.tag, "env": args.env, "B": args.B, "dtype": args.dtype, "kernel": vi.kernel_name,
                      "sweeps": k, "us_per_solve": round(float(np.median(wall)), 2),
                      "kernel_us": round(float(np.median(kern)), 2), "method": args.method,
                      "launches": launches,
                      "updates_per_s": upd / (float(np.median(wall)) * 1e-6),
                      "executed_frac": round(float(gs.mean()) / k, 4),
                      "wall_all": [round(x, 1) for x in wall]}), flush=True)
    vi.close()


if __name__ == "__main__":
    main()
