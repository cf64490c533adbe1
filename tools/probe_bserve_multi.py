"""Debug probe: the batch server past its resident capacity (MGDP_BSERVE=2) against the oracle, per
grid: after one request on a fresh launch, after three on one launch, and with launches."""
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
    vi = mg.ValueIteration(cells, dtype="f32")

    def bad():
        V = vi.values().reshape(B, -1)
        return np.nonzero((V != ov).any(axis=1))[0]

    res = {}
    vi.solve()
    res["one_request"] = bad()[:12].tolist()
    for _ in range(3):
        vi.solve()
    res["three_requests"] = bad()[:12].tolist()
    vi.enable_timing(True)
    vi.solve()
    res["launch"] = bad()[:12].tolist()
    vi.enable_timing(False)
    vi.close()
    os.environ["MGDP_BSERVE_WAIT_PUB"] = "0"
    vi = mg.ValueIteration(cells, dtype="f32")
    vi.solve()
    vi.solve()
    res["no_wait_pub"] = bad()[:12].tolist()
    vi.close()
    os.environ["MGDP_BSERVE_WAIT_PUB"] = "1"
    os.environ["MGDP_BSERVE"] = "1"
    vi = mg.ValueIteration(cells[:cap], dtype="f32")
    vi.solve()
    vi.solve()
    V = vi.values().reshape(cap, -1)
    res["resident_cap"] = np.nonzero((V != ov[:cap]).any(axis=1))[0][:12].tolist()
    vi.close()
    os.environ["MGDP_BSERVE"] = "2"
    os.environ["MGDP_BSERVE_FORCE_MULTI"] = "1"
    vi = mg.ValueIteration(cells[:cap], dtype="f32")
    vi.solve()
    vi.solve()
    V = vi.values().reshape(cap, -1)
    res["multi_kernel_at_cap"] = np.nonzero((V != ov[:cap]).any(axis=1))[0][:12].tolist()
    vi.close()
    vi = mg.ValueIteration(cells[:cap // 2], dtype="f32")
    vi.solve()
    vi.solve()
    V = vi.values().reshape(cap // 2, -1)
    res["multi_kernel_half_cap"] = np.nonzero((V != ov[:cap // 2]).any(axis=1))[0][:12].tolist()
    vi.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
