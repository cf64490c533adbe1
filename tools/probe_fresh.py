"""First solve after a cells load vs the next solve of the same grids (round 6):
wall time of one solve (+ synchronize) and its kernel time (HIP events), for new grids and for the
same grids re-loaded, on one batched BASELINE config.  Prints one JSON line per case."""
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
    ap.add_argument("--B", type=int, default=65536)
    ap.add_argument("--sets", type=int, default=3)
    args = ap.parse_args()
    import torch

    import minigrid_dynamicprogramming_amd as mg
    from minigrid_dynamicprogramming_amd import _lib, gen

    _lib.pin_host_thread(0)
    sets = [gen.generate(args.env, i * args.B, args.B, enc=False, cells=True, agent=False)["cells"] for i in range(args.sets + 1)]
    vi = mg.ValueIteration(sets[0])
    for _ in range(5):
        vi.solve()
    vi.synchronize()

    def timed():
        torch.cuda.synchronize()
        vi.enable_timing(True)
        t = time.perf_counter()
        vi.solve()
        vi.synchronize()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t) * 1e6
        ms, n = vi.kernel_time()
        vi.enable_timing(False)
        return round(wall, 2), round(ms * 1e3, 2), n

    for case in ("new", "same", "device_new"):
        rows = []
        for i in range(1, args.sets + 1):
            c = sets[i] if case != "same" else sets[0]
            if case == "device_new":
                t = torch.from_numpy(np.ascontiguousarray(c)).cuda()
                torch.cuda.synchronize()
                vi.load_device(t.data_ptr())
            else:
                vi.load(c)
            rows.append((timed(), timed(), timed()))
        print(json.dumps({"env": args.env, "B": args.B, "case": case,
                          "first_wall_kern_launches": [r[0] for r in rows], "second": [r[1] for r in rows],
                          "third": [r[2] for r in rows]}), flush=True)
    vi.close()


if __name__ == "__main__":
    main()
