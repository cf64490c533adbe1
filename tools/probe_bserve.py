"""Resident batch server vs a launch per solve, one configuration: wall per solve of each, the
launch's kernel time (HIP events) and the server's GPU-side time per solve (its forwarder's
request-seen -> own exit work done, s_memrealtime; mgdp_vi_serve_clock).  One JSON line."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="MiniGrid-LavaCrossingS11N5-v0")
    ap.add_argument("--B", type=int, default=8192)
    ap.add_argument("--solves", type=int, default=50)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--tag", default="")
    ap.add_argument("--trace", action="store_true",
                    help="trace build (MGDP_BSERVE_TRACE): per-grid start / end after the request, from grid_sweeps()")
    args = ap.parse_args()
    import torch

    import minigrid_dynamicprogramming_amd as mg
    from minigrid_dynamicprogramming_amd import _lib, gen

    _lib.pin_host_thread(0)
    cells = gen.generate(args.env, 0, args.B, enc=False, cells=True, agent=False)["cells"]
    vi = mg.ValueIteration(cells, dtype="f32")
    wall, gpu = [], []
    for _ in range(args.reps):
        vi.enable_timing(False)  # resets the server clock too
        vi.solve()
        t = time.perf_counter()
        for _ in range(args.solves):
            k = vi.solve()
        wall.append((time.perf_counter() - t) * 1e6 / args.solves)
        clk = vi.serve_clock()
        gpu.append(clk["gpu_solve_us"])
    trace = None
    if args.trace:  # the last served solve's per-grid words: start | end << 16, 10 ns ticks
        vi.enable_timing(False)
        vi.solve()
        vi.solve()
        w = vi.grid_sweeps().astype(np.int64) & 0xffffffff
        st, en = (w & 0xffff) * 0.01, (w >> 16) * 0.01
        trace = {"start_us_pcts": [round(float(np.percentile(st, q)), 2) for q in (0, 50, 90, 99, 100)],
                 "end_us_pcts": [round(float(np.percentile(en, q)), 2) for q in (0, 50, 90, 99, 100)]}
    # the server's last request (mgdp_vi_solve_last): its wall, and the launches the clock counted
    vi.enable_timing(False)
    for _ in range(5):
        vi.solve()
    t = time.perf_counter()
    vi.solve(True)
    last_us = (time.perf_counter() - t) * 1e6
    vi.synchronize()
    clk_last = vi.serve_clock()
    vi.enable_timing(True)
    for _ in range(args.solves):
        vi.solve()
    ms, n = vi.kernel_time()
    torch.cuda.synchronize()
    print(json.dumps({"tag": args.tag, "env": args.env, "B": args.B, "sweeps": k,
                      "served_us": round(float(np.median(wall)), 2), "served_gpu_us": round(float(np.median(gpu)), 2),
                      "solves_served": clk["solves"], "launch_kernel_us": round(ms * 1e3 / max(n, 1), 2), "trace": trace,
                      "last_us": round(last_us, 2), "last_launches": clk_last["launches"], "last_solves": clk_last["solves"]}),
          flush=True)
    vi.close()


if __name__ == "__main__":
    main()
