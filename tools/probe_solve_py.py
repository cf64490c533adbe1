"""Lone-grid solve latency from Python (the bench's path) next to the C-ABI probe: per-solve wall
time of ValueIteration.solve() on Empty-16x16 (29 sweeps), and of the raw ctypes call.
MGDP_PROBE_TORCH=1 initialises torch on the device first (as bench.py does), MGDP_PROBE_PIN=0
leaves the thread unpinned (default: pinned to the GPU's NUMA node before the handle exists)."""
import json
import os
import time

import numpy as np

import minigrid_dynamicprogramming_amd as mg


def main():
    if os.environ.get("MGDP_PROBE_TORCH") == "1":
        import torch

        torch.cuda.set_device(0)
    pinned = mg._lib.pin_host_thread(0) if os.environ.get("MGDP_PROBE_PIN", "1") == "1" else 0
    enc, _ = mg.make("MiniGrid-Empty-16x16-v0").generate(seed=0)
    cells = np.ascontiguousarray(enc[:, :, 0].T)[None]
    vi = mg.ValueIteration(cells, gamma=0.99, tol=1e-6, dtype="f32")
    for _ in range(200):
        vi.solve()
    n = 5000
    t = np.empty(n)
    for i in range(n):
        a = time.perf_counter()
        vi.solve()
        t[i] = time.perf_counter() - a
    f = vi.L.mgdp_vi_solve
    args = vi._solve_args
    t2 = np.empty(n)
    for i in range(n):
        a = time.perf_counter()
        f(*args)
        t2[i] = time.perf_counter() - a
    # the same entry point through ctypes.PyDLL: no GIL release / re-acquire around the call
    import ctypes

    pf = ctypes.PyDLL(mg._lib.lib_path()).mgdp_vi_solve
    pf.restype = ctypes.c_int
    t3 = np.empty(n)
    for i in range(n):
        a = time.perf_counter()
        pf(*args)
        t3[i] = time.perf_counter() - a
    for tag, x in (("solve()", t), ("raw ctypes", t2), ("pydll", t3)):
        print(json.dumps({"tag": tag, "pinned": pinned, "torch": os.environ.get("MGDP_PROBE_TORCH") == "1", "sweeps": vi.sweeps, "mean_us": x.mean() * 1e6, "median_us": float(np.median(x)) * 1e6,
                          "p10_us": float(np.percentile(x, 10)) * 1e6, "p90_us": float(np.percentile(x, 90)) * 1e6}))
    vi.close()


if __name__ == "__main__":
    main()
