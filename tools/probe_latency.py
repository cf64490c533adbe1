"""Per-sweep cost vs fixed cost of the single-grid fused solve (kernel time by HIP events)."""
import sys, time, json
import numpy as np
sys.path.insert(0, ".")
import minigrid_dynamicprogramming_amd as mg

env = mg.make(sys.argv[1] if len(sys.argv) > 1 else "MiniGrid-Empty-16x16-v0")
enc, _ = env.generate(seed=0)
out = {}
for ms in (1, 2, 4, 8, 16, 29):
    vi = mg.ValueIteration(enc[None], max_sweeps=ms, dtype="f32")
    for _ in range(20):
        vi.solve()
    vi.enable_timing(True)
    t0 = time.perf_counter()
    n = 200
    for _ in range(n):
        vi.solve()
    el = time.perf_counter() - t0
    kms, launches = vi.kernel_time()
    out[ms] = {"kernel_us": kms * 1000 / launches, "wall_us": el * 1e6 / n, "sweeps": vi.sweeps}
    vi.close()
print(json.dumps(out, indent=1))
