"""Fixed-work timing of the batched DoorKey kernel: run_to(K) on a fresh handle runs exactly K sweeps
of every grid (the k_target loop of fused_fast_dk_soa: the same LDS traffic and arithmetic as the
own-rule loop, without the stop test), so builds that change the loop can be compared per sweep
even when they change the results (MGDP_LIB diagnostic builds).  Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
import minigrid_dynamicprogramming_amd as mg  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "doorkey65536"
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 69
    cells, _ = bench.make_cells(bench.WORKLOADS[name], 0, 1)
    vi = mg.ValueIteration(cells, dtype="f32")
    vi.reset()
    vi.run_to(K)  # warm
    best = None
    for _ in range(3):
        vi.reset()
        vi.enable_timing(True)
        t0 = time.perf_counter()
        vi.run_to(K)
        wall = time.perf_counter() - t0
        ms, n = vi.kernel_time()
        vi.enable_timing(False)
        if best is None or ms < best[0]:
            best = (ms, n, wall)
    print(json.dumps({"workload": name, "K": K, "lib": os.environ.get("MGDP_LIB", "default"),
                      "dk5": os.environ.get("MGDP_DK5", "1"), "kernel_ms": best[0], "launches": best[1],
                      "us_per_sweep": best[0] * 1e3 / K, "wall_ms": best[2] * 1e3}), flush=True)
    vi.close()


if __name__ == "__main__":
    main()
