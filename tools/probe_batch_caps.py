"""Where a batched one-wave solve's time goes: kernel us per solve (HIP events) under max_sweeps caps
(every grid runs min(cap, its own stopping sweep)), so the slope over the caps is the per-sweep cost
of a wave at that occupancy and the intercept the launch's fixed work (cells, topology, exit:
reduction, pi pass, V store).  One JSON line per (env, B)."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="MiniGrid-FourRooms-v0")
    ap.add_argument("--B", type=int, nargs="+", default=[1024, 2048, 4096])
    ap.add_argument("--caps", type=int, nargs="+", default=[1, 2, 4, 8, 16, 24, 0])
    ap.add_argument("--solves", type=int, default=20)
    args = ap.parse_args()
    import minigrid_dynamicprogramming_amd as mg
    from minigrid_dynamicprogramming_amd import _lib, gen

    _lib.pin_host_thread(0)
    for B in args.B:
        cells = gen.generate(args.env, 0, B, enc=False, cells=True, agent=False)["cells"]
        row = {"env": args.env, "B": B, "caps": {}}
        for cap in args.caps:
            kw = {"max_sweeps": cap} if cap > 0 else {}
            vi = mg.ValueIteration(cells, dtype="f32", **kw)
            for _ in range(3):
                k = vi.solve()
            vi.enable_timing(True)
            for _ in range(args.solves):
                k = vi.solve()
            ms, n = vi.kernel_time()
            gs = vi.grid_sweeps()
            row["caps"][str(cap)] = {"k": int(k), "kernel_us": round(ms * 1e3 / max(n, 1), 2),
                                     "kernel_us_per_solve": round(ms * 1e3 / args.solves, 2), "launches": n,
                                     "mean_grid_sweeps": round(float(np.mean(gs)), 2), "kernel": vi.kernel_name}
            vi.close()
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
