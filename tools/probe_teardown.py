"""Where the lone-grid bench's fixed per-region cost goes: K served solves, then the end-of-region
teardown (vi.synchronize(): quit word + stream drain, then torch.cuda.synchronize()), timed
separately over many regions.  Run under different host-wait settings (ROC_ACTIVE_WAIT_TIMEOUT,
--spin: hipSetDeviceFlags(hipDeviceScheduleSpin) before torch touches the device)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import minigrid_dynamicprogramming_amd as mg  # noqa: E402


def main():
    if "--spin" in sys.argv:
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        rc = hip.hipSetDeviceFlags(ctypes.c_uint(1))  # hipDeviceScheduleSpin
        print(f"hipSetDeviceFlags(spin) -> {rc}", file=sys.stderr)
    enc, _ = mg.make("MiniGrid-Empty-16x16-v0").generate(seed=0)
    cells = np.ascontiguousarray(enc[:, :, 0].T)[None]
    torch.cuda.set_device(0)
    vi = mg.ValueIteration(cells, gamma=0.99, tol=1e-6, dtype="f32")
    for _ in range(50):
        vi.solve()
    timing = "--timing" in sys.argv
    vi.enable_timing(timing)
    R, K = 40, 20
    rows = {"prime": [], "solves": [], "vi_sync": [], "dev_sync": [], "dev_sync_idle": []}
    for _ in range(R):
        torch.cuda.synchronize()
        a = time.perf_counter()
        vi.solve()
        b = time.perf_counter()
        for _ in range(K):
            vi.solve()
        c = time.perf_counter()
        vi.synchronize()
        d = time.perf_counter()
        torch.cuda.synchronize()
        e = time.perf_counter()
        torch.cuda.synchronize()
        f = time.perf_counter()
        rows["prime"].append(b - a)
        rows["solves"].append((c - b) / K)
        rows["vi_sync"].append(d - c)
        rows["dev_sync"].append(e - d)
        rows["dev_sync_idle"].append(f - e)
    out = {k: {"median_us": float(np.median(v)) * 1e6, "p10_us": float(np.percentile(v, 10)) * 1e6,
               "p90_us": float(np.percentile(v, 90)) * 1e6} for k, v in rows.items()}
    out["env"] = {k: os.environ.get(k) for k in ("ROC_ACTIVE_WAIT_TIMEOUT",)}
    out["timing"] = timing
    out["spin"] = "--spin" in sys.argv
    print(json.dumps(out))
    vi.close()


if __name__ == "__main__":
    main()
