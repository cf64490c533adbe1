"""Debug probe: what differs in the grids the multi-grid batch server gets wrong."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    os.environ["MGDP_BSERVE"] = "2"
    import torch

    import minigrid_dynamicprogramming_amd as mg
    from oracle import oracle
    from tests.test_gpu_wave2 import random_grids

    cus = torch.cuda.get_device_properties(0).multi_processor_count
    cap = 32 * cus
    B = cap + 1
    cells = random_grids(B, 9, 7, seed=7, goals=2)
    o = oracle.value_iteration(0, cells, dtype="f32", nthreads=16, fixed_point=True)
    ov = o["V"].reshape(B, -1)
    op = o["pi"].reshape(B, -1)
    vi = mg.ValueIteration(cells, dtype="f32")
    vi.solve()
    V = vi.values().reshape(B, -1)
    P = vi.policy().reshape(B, -1)
    bad = np.nonzero((V != ov).any(axis=1))[0]
    if os.environ.get("MGDP_LIB", "").endswith("_dbg.so"):
        w = vi.grid_sweeps()
        print(json.dumps({"bad_wg": [int(w[g] & 0xfffff) for g in bad[:20]], "bad_iter": [int(w[g] >> 20) for g in bad[:20]],
                          "iters": np.bincount((w >> 20).astype(np.int64)).tolist(),
                          "wg_of_iter1": [int(x & 0xfffff) for x in w[(w >> 20) == 1][:8]]}))
    print(json.dumps({"n_bad": int(len(bad)), "pi_bad": int((P != op).any(axis=1).sum()), "dv": vi.dv}))
    for g in bad[:3]:
        d = np.nonzero(V[g] != ov[g])[0]
        print(json.dumps({"g": int(g), "states": d.tolist(), "gpu": V[g][d].tolist(), "oracle": ov[g][d].tolist(),
                          "cells": cells[g].tolist(), "pi_diff": np.nonzero(P[g] != op[g])[0].tolist()}))


if __name__ == "__main__":
    main()
