"""Mixed wave counts (MGDP_MIX=1, round 5): once a handle's grids have been solved, the learned
dispatch order puts the grids that ran longest first and the first nmix workgroups sweep them on two
waves (fused_wave2n_xyd) while the rest stay on one (fused_wave2_xyd) -- against the oracle's
literal global loop: sweeps, V, pi and per-grid executed sweeps bit for bit over repeated solves,
every P = 2..6 class, every split fraction (0: all grids on two waves), run_to caps, and batches past
the resident capacity (the in-launch reduction for any B, MGDP_GK=1)."""
import numpy as np
import pytest

import minigrid_dynamicprogramming_amd as mg
from minigrid_dynamicprogramming_amd import gen
from oracle import oracle
from tests.test_gpu_wave2 import random_grids

pytestmark = pytest.mark.gpu


def _check(vi, o, grid_sweeps=True):
    np.testing.assert_array_equal(vi.values(), o["V"])
    np.testing.assert_array_equal(vi.policy(), o["pi"])
    if grid_sweeps:
        np.testing.assert_array_equal(vi.grid_sweeps(), o["grid_sweeps"])


@pytest.mark.parametrize("frac", ["0", "0.5", "0.75", "1"])
@pytest.mark.parametrize("env_id,B", [("MiniGrid-LavaCrossingS11N5-v0", 2048), ("MiniGrid-FourRooms-v0", 1024),
                                      ("MiniGrid-Empty-16x16-v0", 1100)])
def test_mixed_waves_match_oracle(env_id, B, frac, monkeypatch):
    monkeypatch.setenv("MGDP_MIX", "1")
    monkeypatch.setenv("MGDP_MIX_FRAC", frac)
    cells = gen.generate(env_id, 3, B, enc=False, cells=True, agent=False)["cells"]
    o = oracle.value_iteration(0, cells, dtype="f32", nthreads=16, fixed_point=True)
    vi = mg.ValueIteration(cells, dtype="f32")
    try:
        assert vi.variant == "mix"
        for _ in range(3):  # solve 1: one wave per grid; solves 2, 3: the learned split
            assert vi.solve() == o["sweeps"]
            _check(vi, o)
    finally:
        vi.close()


@pytest.mark.parametrize("W,H", [(11, 11), (9, 20), (16, 16), (21, 14), (19, 19)])
def test_mixed_waves_random_rooms(W, H, monkeypatch):
    """Random rooms of every P class (2..6 blocks of 64 cells), goals near the block and wave edges."""
    monkeypatch.setenv("MGDP_MIX", "1")
    monkeypatch.setenv("MGDP_MIX_FRAC", "0.6")
    cells = random_grids(1030, W, H, seed=W * 31 + H, goals=1 + (W % 3))
    o = oracle.value_iteration(0, cells, dtype="f32", nthreads=16, fixed_point=True)
    vi = mg.ValueIteration(cells, dtype="f32")
    try:
        assert vi.variant == "mix"
        for _ in range(2):
            assert vi.solve() == o["sweeps"]
            _check(vi, o)
    finally:
        vi.close()


@pytest.mark.parametrize("ms", [1, 7, 20])
def test_mixed_waves_caps_and_protocol(ms, monkeypatch):
    """max_sweeps caps, and run_local + run_to (the protocol's launches) on the learned split."""
    monkeypatch.setenv("MGDP_MIX", "1")
    monkeypatch.setenv("MGDP_MIX_FRAC", "0.5")
    cells = gen.generate("MiniGrid-LavaCrossingS11N5-v0", 11, 1500, enc=False, cells=True, agent=False)["cells"]
    oc = oracle.value_iteration(0, cells, dtype="f32", nthreads=16, max_sweeps=ms)
    vi = mg.ValueIteration(cells, dtype="f32", max_sweeps=ms)
    try:
        for _ in range(2):
            assert vi.solve() == oc["sweeps"] == ms
            _check(vi, oc, grid_sweeps=False)
    finally:
        vi.close()
    o = oracle.value_iteration(0, cells, dtype="f32", nthreads=16)
    vi = mg.ValueIteration(cells, dtype="f32")
    try:
        vi.solve()  # learn the order
        vi.reset()
        k = vi.run_local()
        assert k == o["sweeps"]
        vi.reset()
        vi.run_to(k - 3)
        dv = vi.run_to(k)
        vi.finish(k, dv)
        _check(vi, o, grid_sweeps=False)
    finally:
        vi.close()


@pytest.mark.parametrize("gk", ["1", "2", "0"])
def test_inlaunch_reduction_past_capacity(gk, monkeypatch):
    """LavaS11N5 x 20000 (past the one-wave kernel's 8192 resident grids): the in-launch reduction for
    any B (MGDP_GK=1), the resident-only rule (2, the default: the reduce kernel here) and the reduce
    kernel (0) agree."""
    monkeypatch.setenv("MGDP_GK", gk)
    cells = gen.generate("MiniGrid-LavaCrossingS11N5-v0", 5, 20000, enc=False, cells=True, agent=False)["cells"]
    o = oracle.value_iteration(0, cells, dtype="f32", nthreads=16, fixed_point=True)
    vi = mg.ValueIteration(cells, dtype="f32")
    try:
        for _ in range(2):
            assert vi.solve() == o["sweeps"]
            assert vi.dv == o["dv"]
            _check(vi, o)
    finally:
        vi.close()
