"""Host cost of launch timing on batched solves: wall time per solve of the BASELINE batches with
the library's HIP-event launch timing on vs off (alternating blocks of solves on one handle), and
the kernel time the events report.  One JSON line per workload."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import minigrid_dynamicprogramming_amd as mg
    from minigrid_dynamicprogramming_amd import _lib, gen

    _lib.pin_host_thread(0)
    for env_id, B in [("MiniGrid-FourRooms-v0", 4096), ("MiniGrid-LavaCrossingS11N5-v0", 65536),
                      ("MiniGrid-LavaCrossingS11N5-v0", 8192)]:
        cells = gen.generate(env_id, 0, B, enc=False, cells=True, agent=False)["cells"]
        vi = mg.ValueIteration(cells, dtype="f32")
        res = {True: [], False: []}
        kern = []
        for rep in range(6):
            for on in (True, False):
                vi.enable_timing(on)
                vi.solve()
                torch.cuda.synchronize()
                t = time.perf_counter()
                for _ in range(20):
                    vi.solve()
                res[on].append((time.perf_counter() - t) * 1e6 / 20)
                if on:
                    ms, n = vi.kernel_time()
                    kern.append(ms * 1e3 / max(n, 1))
        vi.close()
        print(json.dumps({"env": env_id, "B": B, "us_per_solve_timing_on": round(float(np.median(res[True])), 2),
                          "us_per_solve_timing_off": round(float(np.median(res[False])), 2),
                          "kernel_us": round(float(np.median(kern)), 2),
                          "on_all": [round(x, 1) for x in res[True]], "off_all": [round(x, 1) for x in res[False]]}),
              flush=True)


if __name__ == "__main__":
    main()
