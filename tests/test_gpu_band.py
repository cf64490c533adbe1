"""Deterministic XYD grids on fused_band_xyd (round 5: one wave per grid, lane b*W + x owns column x
of band b, north / south fronts in registers and two ds_bpermute values across band edges, east /
west fronts by DPP, no LDS tile), batched (MGDP_BAND=1) and as the served lone grid
(MGDP_SERVE_BAND=1), against the oracle's literal global loop: sweeps, V, pi (and the served dV)
bit for bit, fp32 and fp64; every rows-per-band class HB = 1..8, walkable cells next to band
edges, max_sweeps caps, the protocol's run_local + run_to, and new grids handed to a resident
server."""
import numpy as np
import pytest

import minigrid_dynamicprogramming_amd as mg
from minigrid_dynamicprogramming_amd import gen
from oracle import oracle
from tests.test_gpu_wave2 import random_grids

pytestmark = pytest.mark.gpu

# (W, H) -> HB = ceil(H / (64 // W)), every class 1..8: 1 (5x5, 9x7), 2 (11x10), 3 (11x11 LavaS11N5,
# 9x20), 4 (16x16, 13x13, 21x12), 5 (16x20), 6 (40x6), 7 (19x19 FourRooms), 8 (32x16); 22x22 (HB 11)
# stays on fused_wave2_xyd
SHAPES = [(5, 5), (9, 7), (11, 10), (11, 11), (9, 20), (16, 16), (13, 13), (21, 12), (16, 20), (40, 6), (19, 19),
          (32, 16), (22, 22)]


def band_rows(W, H):
    return -(-H // (64 // W)) if W <= 64 else 0


@pytest.mark.parametrize("dtype", ["f32", "f64"])
@pytest.mark.parametrize("W,H", SHAPES)
def test_batched_band_matches_oracle(W, H, dtype, monkeypatch):
    monkeypatch.setenv("MGDP_BAND", "1")
    cells = random_grids(41, W, H, seed=W * 7 + H, goals=1 + (H % 3))
    vi = mg.ValueIteration(cells, dtype=dtype)
    try:
        assert vi.variant == ("band" if 1 <= band_rows(W, H) <= 8 else "wave2")
        k = vi.solve()
        o = oracle.value_iteration(0, cells, dtype=dtype)
        assert k == o["sweeps"]
        np.testing.assert_array_equal(vi.values(), o["V"])
        np.testing.assert_array_equal(vi.policy(), o["pi"])
    finally:
        vi.close()


@pytest.mark.parametrize("env_id,B", [("MiniGrid-FourRooms-v0", 4096), ("MiniGrid-LavaCrossingS11N5-v0", 9000),
                                      ("MiniGrid-Empty-16x16-v0", 700)])
def test_batched_band_baseline_families(env_id, B, monkeypatch):
    """The BASELINE families at scale: in-launch reduction (resident) and the reduce kernel (9000
    LavaS11N5 grids), the learned dispatch order on the second and third solve."""
    monkeypatch.setenv("MGDP_BAND", "1")
    cells = gen.generate(env_id, 0, B, enc=False, cells=True, agent=False)["cells"]
    o = oracle.value_iteration(0, cells, dtype="f32", nthreads=16, fixed_point=True)
    vi = mg.ValueIteration(cells, dtype="f32")
    try:
        assert vi.variant == "band"
        for _ in range(3):
            assert vi.solve() == o["sweeps"]
            np.testing.assert_array_equal(vi.values(), o["V"])
            np.testing.assert_array_equal(vi.policy(), o["pi"])
            np.testing.assert_array_equal(vi.grid_sweeps(), o["grid_sweeps"])
    finally:
        vi.close()


@pytest.mark.parametrize("ms", [1, 2, 5, 13])
def test_batched_band_caps_and_protocol(ms, monkeypatch):
    monkeypatch.setenv("MGDP_BAND", "1")
    cells = random_grids(64, 19, 19, seed=ms, goals=2)
    o = oracle.value_iteration(0, cells, dtype="f32", max_sweeps=ms)
    r = mg.value_iteration(cells, dtype="f32", max_sweeps=ms)
    assert r.sweeps == o["sweeps"] == ms
    np.testing.assert_array_equal(r.V, o["V"])
    np.testing.assert_array_equal(r.pi, o["pi"])
    # run_local, a fresh run_to to a fixed sweep, then on to K from HBM
    o = oracle.value_iteration(0, cells, dtype="f32")
    vi = mg.ValueIteration(cells, dtype="f32")
    try:
        vi.reset()
        k = vi.run_local()
        assert k == o["sweeps"]
        vi.reset()
        vi.run_to(ms)
        dv = vi.run_to(k)
        vi.finish(k, dv)
        np.testing.assert_array_equal(vi.values(), o["V"])
        np.testing.assert_array_equal(vi.policy(), o["pi"])
    finally:
        vi.close()


@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_served_band_lone_grids(dtype, monkeypatch):
    """The resident server on one band wave: Empty-16 (the headline grid), FourRooms and LavaS11N5
    seeds and random rooms handed over as new grids between solves; sweeps, dV, V and pi."""
    monkeypatch.setenv("MGDP_PERSISTENT", "1")
    monkeypatch.setenv("MGDP_SERVE_BAND", "1")
    grids = []
    for env_id, n in (("MiniGrid-Empty-16x16-v0", 1), ("MiniGrid-FourRooms-v0", 3), ("MiniGrid-LavaCrossingS11N5-v0", 3)):
        grids += list(gen.generate(env_id, 5, n, enc=False, cells=True, agent=False)["cells"])
    by_shape = {}
    for g in grids + list(random_grids(4, 16, 16, seed=3, goals=2)) + list(random_grids(3, 19, 19, seed=4)):
        by_shape.setdefault(g.shape, []).append(g)
    for shape, gs in by_shape.items():
        vi = mg.ValueIteration(gs[0][None], dtype=dtype)
        try:
            assert vi.persistent and vi.variant == "serve_band"
            for rep in range(2):
                for g in gs:
                    vi.load(g[None])
                    k = vi.solve()
                    o = oracle.value_iteration(0, g[None], dtype=dtype)
                    assert k == o["sweeps"] and vi.dv == o["dv"]
                    if rep:
                        np.testing.assert_array_equal(vi.values(), o["V"])
                        np.testing.assert_array_equal(vi.policy(), o["pi"])
        finally:
            vi.close()


def test_served_band_headline_repeated_and_capped(monkeypatch):
    monkeypatch.setenv("MGDP_PERSISTENT", "1")
    monkeypatch.setenv("MGDP_SERVE_BAND", "1")
    enc, _ = mg.make("MiniGrid-Empty-16x16-v0").generate(seed=0)
    g = np.ascontiguousarray(enc[..., 0].T)[None]
    vi = mg.ValueIteration(g, dtype="f32")
    try:
        for _ in range(200):
            assert vi.solve() == 29
        o = oracle.value_iteration(0, g, dtype="f32")
        np.testing.assert_array_equal(vi.values(), o["V"])
        np.testing.assert_array_equal(vi.policy(), o["pi"])
    finally:
        vi.close()
    for ms in (1, 3, 28):
        vi = mg.ValueIteration(g, dtype="f32", max_sweeps=ms)
        try:
            assert vi.solve() == ms
            o = oracle.value_iteration(0, g, dtype="f32", max_sweeps=ms)
            np.testing.assert_array_equal(vi.values(), o["V"])
            np.testing.assert_array_equal(vi.policy(), o["pi"])
        finally:
            vi.close()
