# (Measured and dropped: the one-launch solve is no longer in the library -- polling one launch-wide word
#  serialised the grids, 104 vs 46 us at 64 FourRooms grids; record of profiles/r02_gsync/.)
"""One-launch solve (gsync) on FourRooms x B: where it aborts, and its time vs the two-launch chain."""
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import minigrid_dynamicprogramming_amd as mg  # noqa: E402
from minigrid_dynamicprogramming_amd import gen  # noqa: E402

os.environ["MGDP_GSYNC_DEBUG"] = "1"
for B in (600, 700, 768, 896):
    cells = gen.generate("MiniGrid-FourRooms-v0", 0, B, enc=False, cells=True, agent=False)["cells"]
    vi = mg.ValueIteration(cells, dtype="f32")
    print(B, [vi.solve() for _ in range(1)], flush=True)
    vi.close()
os.environ["MGDP_GSYNC_DEBUG"] = "0"
for B in (64, 256, 512):
    cells = gen.generate("MiniGrid-FourRooms-v0", 0, B, enc=False, cells=True, agent=False)["cells"]
    for g in ("1", "0", "1", "0"):
        os.environ["MGDP_GSYNC"] = g
        vi = mg.ValueIteration(cells, dtype="f32")
        for _ in range(5):
            vi.solve()
        n = 200
        t = time.perf_counter()
        for _ in range(n):
            k = vi.solve()
        dt = (time.perf_counter() - t) / n
        vi.close()
        print(B, "gsync", g, k, "%.1f us/solve" % (dt * 1e6), flush=True)
