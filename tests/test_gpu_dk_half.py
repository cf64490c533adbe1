"""Batched DoorKey grids on fused_dk_half (each cell's 16 states over two threads split by
has_key, plane stride compiled per 64-cell size class: tags -501 .. -508) against the oracle and
against the one-thread-per-cell loop (MGDP_DK_HALF=0): sweeps, V and pi bit-exact at a size in
every class, fp32 and fp64, max_sweeps caps, and the two-launch protocol (run_local, then run_to
continuing from V in HBM)."""
import numpy as np
import pytest

import minigrid_dynamicprogramming_amd as mg
from minigrid_dynamicprogramming_amd.envs import DoorKeyEnv
from oracle import oracle

pytestmark = pytest.mark.gpu


def doorkey_cells(size, n, seed0=0):
    env = DoorKeyEnv(size=size)
    return np.stack([np.ascontiguousarray(env.generate(seed=seed0 + s)[0][..., 0].T) for s in range(n)]).astype(np.uint8)


def solve(cells, dtype, half, monkeypatch, **kw):
    monkeypatch.setenv("MGDP_DK_HALF", half)
    return mg.value_iteration(cells, model="doorkey", dtype=dtype, **kw)


# HW = size^2 cells: 25 (64-cell class), 64, 100 -> 128, 196 -> 256, 256, 324 -> 384, 400 -> 448, 484 -> 512
@pytest.mark.parametrize("size", [5, 8, 10, 14, 16, 18, 20, 22])
@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_dk_half_sizes_vs_oracle(size, dtype, monkeypatch):
    cells = doorkey_cells(size, 9, seed0=size)
    o = oracle.value_iteration(1, cells, dtype=dtype)
    r = solve(cells, dtype, "1", monkeypatch)
    assert r.sweeps == o["sweeps"]
    np.testing.assert_array_equal(r.V, o["V"])
    np.testing.assert_array_equal(r.pi, o["pi"])
    r0 = solve(cells, dtype, "0", monkeypatch)
    assert r0.sweeps == r.sweeps
    np.testing.assert_array_equal(r0.V, r.V)
    np.testing.assert_array_equal(r0.pi, r.pi)


@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_dk_half_max_sweeps_caps(dtype, monkeypatch):
    cells = doorkey_cells(16, 5, seed0=3)
    for ms in (1, 2, 3, 17):
        o = oracle.value_iteration(1, cells, dtype=dtype, max_sweeps=ms)
        r = solve(cells, dtype, "1", monkeypatch, max_sweeps=ms)
        assert r.sweeps == o["sweeps"] == ms
        np.testing.assert_array_equal(r.V, o["V"])
        np.testing.assert_array_equal(r.pi, o["pi"])


def test_dk_half_protocol_continuation(monkeypatch):
    # run_local stops each grid at its own sweep; run_to continues every grid from V in HBM
    monkeypatch.setenv("MGDP_DK_HALF", "1")
    cells = doorkey_cells(8, 12, seed0=40)
    o = oracle.value_iteration(1, cells, dtype="f32")
    vi = mg.ValueIteration(cells, model="doorkey", dtype="f32")
    try:
        vi.reset()
        k = vi.run_local()
        assert k == o["sweeps"]
        vi.run_to(k)
        vi.finish(k, 0.0)
        np.testing.assert_array_equal(vi.values(), o["V"])
        np.testing.assert_array_equal(vi.policy(), o["pi"])
        vi.reset()
        vi.run_to(5)  # fresh loop to a fixed sweep, then continue to K from HBM
        vi.run_to(k)
        vi.finish(k, 0.0)
        np.testing.assert_array_equal(vi.values(), o["V"])
        np.testing.assert_array_equal(vi.policy(), o["pi"])
    finally:
        vi.close()


@pytest.mark.parametrize("persistent", ["0", "1"])
@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_dk_half_lone_grid_served_and_launched(persistent, dtype, monkeypatch):
    # a lone grid on the split loop: the resident server (grid per request included) or one launch
    monkeypatch.setenv("MGDP_PERSISTENT", persistent)
    monkeypatch.setenv("MGDP_DK_HALF", "1")
    for size in (6, 16, 22):
        cells = doorkey_cells(size, 4, seed0=100 + size)
        vi = mg.ValueIteration(cells[:1], model="doorkey", dtype=dtype)
        try:
            assert vi.persistent == (persistent == "1")
            for i in range(len(cells)):
                vi.load(cells[i:i + 1])
                k = vi.solve()
                o = oracle.value_iteration(1, cells[i:i + 1], dtype=dtype)
                assert k == o["sweeps"]
                if i % 2:
                    r = vi.result()
                    np.testing.assert_array_equal(r.V, o["V"])
                    np.testing.assert_array_equal(r.pi, o["pi"])
        finally:
            vi.close()
