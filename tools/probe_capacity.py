"""The capacity case of tests/test_gpu_fixedpoint.py (one-wave P = 1 grids: the resident capacity
+ delta, next to a resident lone-grid server) timed under the knobs named on the command line
(KEY=VALUE ...), one JSON line: median us per solve with the in-launch reduction (GK) and with the
reduce kernel (MGDP_GK=0)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    kv = dict(a.split("=", 1) for a in sys.argv[1:] if "=" in a)
    os.environ.update(kv)
    import torch

    import minigrid_dynamicprogramming_amd as mg
    from tests.test_gpu_wave2 import random_grids

    cap = 32 * torch.cuda.get_device_properties(0).multi_processor_count
    out = {"knobs": kv}
    enc, _ = mg.make("MiniGrid-Empty-16x16-v0").generate(seed=0)
    os.environ["MGDP_SERVE_IDLE_US"] = "500000"
    lone = mg.ValueIteration(np.ascontiguousarray(enc[..., 0].T)[None], dtype="f32")
    del os.environ["MGDP_SERVE_IDLE_US"]
    lone.solve()
    for delta in (-1, 0, 1):
        cells = random_grids(cap + delta, 9, 7, seed=7, goals=2)
        res = {}
        for gk in ("1", "0"):
            os.environ["MGDP_GK"] = gk
            vi = mg.ValueIteration(cells, dtype="f32")
            ts = []
            for _ in range(5):
                lone.solve()
                vi.solve()
                t = time.perf_counter()
                for _ in range(5):
                    vi.solve()
                ts.append((time.perf_counter() - t) / 5 * 1e6)
            res["gk" + gk] = round(float(np.median(ts)), 2)
            vi.close()
        out[str(delta)] = res
    lone.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
