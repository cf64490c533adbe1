"""Per-sweep cost of the lone grid's stop test: the fused launch (MGDP_PERSISTENT=0) run with the
rule (run_local: ballot + flag byte + read each sweep) against the same 29 sweeps with a fixed
target (run_to from V_0: no flags), kernel durations from the library's HIP events."""
import json
import os
import sys

os.environ["MGDP_PERSISTENT"] = "0"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import minigrid_dynamicprogramming_amd as mg  # noqa: E402


def main():
    enc, _ = mg.make("MiniGrid-Empty-16x16-v0").generate(seed=0)
    cells = np.ascontiguousarray(enc[:, :, 0].T)[None]
    torch.cuda.set_device(0)
    vi = mg.ValueIteration(cells, dtype="f32")
    out = {}
    for mode in ("local", "fixed29", "local", "fixed29"):
        for _ in range(20):
            vi.reset()
            k = vi.run_local() if mode == "local" else (vi.run_to(29), 29)[1]
        vi.enable_timing(True)
        n = 200
        for _ in range(n):
            vi.reset()
            k = vi.run_local() if mode == "local" else (vi.run_to(29), 29)[1]
        ms, launches = vi.kernel_time()
        vi.enable_timing(False)
        out.setdefault(mode, []).append({"sweeps": k, "kernel_us": ms * 1000.0 / launches, "launches": launches})
    print(json.dumps(out))
    vi.close()


if __name__ == "__main__":
    main()
