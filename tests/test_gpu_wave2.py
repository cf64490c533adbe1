"""The one-wave-per-grid batched XYD solver (fused_wave2_xyd: P = ceil(W*H/64) cells per lane,
DPP east/west fronts, one N/S tile) against the oracle on random closed-border grids of every
P it serves (1..8), square and not, odd and even widths, lava and several goals, both dtypes;
the in-kernel (B <= 512) and separate-kernel reductions; and a run_to continuation."""
import numpy as np
import pytest

import minigrid_dynamicprogramming_amd as mg
from oracle import oracle

pytestmark = pytest.mark.gpu


def random_grids(n, W, H, seed, goals=1):
    rng = np.random.default_rng(seed)
    out = np.full((n, H, W), 2, np.uint8)
    for i in range(n):
        out[i, 1:-1, 1:-1] = rng.choice(np.array([1, 1, 1, 1, 2, 9, 3], np.uint8), size=(H - 2, W - 2))
        for _ in range(goals):
            out[i, rng.integers(1, H - 1), rng.integers(1, W - 1)] = 8
    return out


SHAPES = [(5, 5), (9, 7), (10, 12), (13, 13), (16, 16), (15, 21), (19, 19), (21, 21), (23, 22)]


@pytest.mark.parametrize("dtype", ["f32", "f64"])
@pytest.mark.parametrize("W,H", SHAPES)
def test_wave2_matches_oracle(W, H, dtype):
    cells = random_grids(37, W, H, seed=W * 31 + H, goals=1 + (W % 3))
    r = mg.value_iteration(cells, dtype=dtype)
    o = oracle.value_iteration(0, cells, dtype=dtype)
    assert r.sweeps == o["sweeps"]
    np.testing.assert_array_equal(r.pi, o["pi"])
    np.testing.assert_array_equal(r.V, o["V"])


def test_wave2_large_batch_separate_reduce():
    cells = random_grids(600, 11, 11, seed=5)
    r = mg.value_iteration(cells, dtype="f32")
    o = oracle.value_iteration(0, cells, dtype="f32")
    assert r.sweeps == o["sweeps"]
    np.testing.assert_array_equal(r.pi, o["pi"])
    np.testing.assert_array_equal(r.V, o["V"])


def test_wave2_max_sweeps_cap_and_continuation():
    # tol below any |dV|: every grid stops at the cap in run_local; grids converging at different
    # sweeps (the random batches above) exercise run_to's restart from HBM (k > 0)
    cells = random_grids(9, 16, 16, seed=11)
    r = mg.value_iteration(cells, dtype="f64", tol=1e-300, max_sweeps=10)
    o = oracle.value_iteration(0, cells, dtype="f64", tol=1e-300, max_sweeps=10)
    assert r.sweeps == o["sweeps"] == 10 and not r.converged
    np.testing.assert_array_equal(r.pi, o["pi"])
    np.testing.assert_array_equal(r.V, o["V"])


# Two waves per grid (fused_wave2n_xyd): P = ceil(W*H/64) >= 3 blocks split over two waves (PW =
# ceil(P/2), idle blocks past the grid), the wave boundary's east / west values and the stop flags
# through LDS.  MGDP_WAVE2N=1 turns it on (off by default: measured slower).
SHAPES_2N = [(13, 13), (16, 16), (15, 21), (19, 19), (21, 21), (23, 22)]


@pytest.mark.parametrize("dtype", ["f32", "f64"])
@pytest.mark.parametrize("W,H", SHAPES_2N)
def test_wave2n_matches_oracle(W, H, dtype, monkeypatch):
    monkeypatch.setenv("MGDP_WAVE2N", "1")
    cells = random_grids(37, W, H, seed=W * 17 + H, goals=1 + (H % 3))
    r = mg.value_iteration(cells, dtype=dtype)
    o = oracle.value_iteration(0, cells, dtype=dtype)
    assert r.sweeps == o["sweeps"]
    np.testing.assert_array_equal(r.pi, o["pi"])
    np.testing.assert_array_equal(r.V, o["V"])


@pytest.mark.parametrize("B", [600, 4096])
def test_wave2n_batches_and_reductions(B, monkeypatch):
    # 600 grids: the in-launch tree; 4096 FourRooms-sized grids: not all resident, the reduce kernel
    monkeypatch.setenv("MGDP_WAVE2N", "1")
    cells = random_grids(B, 19, 19, seed=B, goals=2)
    r = mg.value_iteration(cells, dtype="f32")
    o = oracle.value_iteration(0, cells, dtype="f32", nthreads=8)
    assert r.sweeps == o["sweeps"]
    np.testing.assert_array_equal(r.pi, o["pi"])
    np.testing.assert_array_equal(r.V, o["V"])


def test_wave2n_cap_and_continuation(monkeypatch):
    # every grid stops at the cap in run_local (no exact fixed point): run_to continues from HBM
    # on the two-wave path with the tile parity restarted at an even / odd k
    monkeypatch.setenv("MGDP_WAVE2N", "1")
    cells = random_grids(9, 19, 19, seed=12)
    for cap in (9, 10):
        r = mg.value_iteration(cells, dtype="f64", tol=1e-300, max_sweeps=cap)
        o = oracle.value_iteration(0, cells, dtype="f64", tol=1e-300, max_sweeps=cap)
        assert r.sweeps == o["sweeps"] == cap and not r.converged
        np.testing.assert_array_equal(r.pi, o["pi"])
        np.testing.assert_array_equal(r.V, o["V"])
    vi = mg.ValueIteration(cells, dtype="f32")
    vi.reset()
    vi.run_to(7)  # fresh loop to an odd sweep, then on to 13 from HBM
    vi.run_to(13)
    vi.finish(13, 0.0)
    o = oracle.value_iteration(0, cells, dtype="f32", tol=-1.0, max_sweeps=13)
    np.testing.assert_array_equal(vi.values(), o["V"])
    np.testing.assert_array_equal(vi.policy(), o["pi"])
    vi.close()
