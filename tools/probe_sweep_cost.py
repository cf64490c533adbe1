"""Per-sweep cost of the single-grid fused loop: the local-rule loop (solve) against the fixed-count
loop (run_to, no convergence flags), by HIP-event kernel time; one fused launch per call."""
import os
import sys
import json
import time

os.environ["MGDP_PERSISTENT"] = "0"
sys.path.insert(0, ".")
import minigrid_dynamicprogramming_amd as mg

env = mg.make(sys.argv[1] if len(sys.argv) > 1 else "MiniGrid-Empty-16x16-v0")
enc, _ = env.generate(seed=0)
vi = mg.ValueIteration(enc[None], dtype="f32")
out = {}


def timed(fn, n=300):
    for _ in range(20):
        fn()
    vi.enable_timing(True)
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    el = time.perf_counter() - t0
    ms, launches = vi.kernel_time()
    vi.enable_timing(False)
    return {"kernel_us": ms * 1000 / max(launches, 1), "launches_per_call": launches / n, "wall_us": el * 1e6 / n}


out["solve_local"] = timed(vi.solve)
for k in (1, 29, 58, 116):
    def f(k=k):
        vi.reset()
        vi.run_to(k)
    out[f"run_to_{k}"] = timed(f)
vi.close()
print(json.dumps(out, indent=1))
