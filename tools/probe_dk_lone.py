"""Lone DoorKey-16 solve time (resident server) with the has_key split on / off, fp32 and fp64."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import minigrid_dynamicprogramming_amd as mg  # noqa: E402

env = mg.make("MiniGrid-DoorKey-16x16-v0")
cells = np.ascontiguousarray(env.generate(seed=0)[0][..., 0].T)[None].astype(np.uint8)
out = {}
for dtype in ("f32", "f64"):
    for half in ("0", "1"):
        os.environ["MGDP_DK_HALF"] = half
        vi = mg.ValueIteration(cells, model="doorkey", dtype=dtype)
        for _ in range(30):
            vi.solve()
        n = 400
        t = time.perf_counter()
        for _ in range(n):
            k = vi.solve()
        dt = (time.perf_counter() - t) / n
        vi.close()
        out[f"{dtype}/half{half}"] = {"us_per_solve": dt * 1e6, "sweeps": k,
                                      "updates_per_s": cells.size * 16 * 5 * k / dt}
        print(dtype, half, "%.2f us" % (dt * 1e6), k, "%.3g upd/s" % out[f"{dtype}/half{half}"]["updates_per_s"], flush=True)
print(json.dumps(out))
