"""Batched DoorKey grids of width 16 on fused_dk_rows (round 5: whole grid rows per 16 lanes, DPP
east / west fronts, two conflict-free LDS planes, the stop test before the next sweep's arithmetic)
against the oracle's literal global Jacobi loop and against the round-4 loop (MGDP_DK_ROWS=0,
fused_fast_dk_soa): global sweep count, V and pi bit-exact, fp32 and fp64.  Covers the
reference-generated DoorKey-16 grids (BASELINE config 5's family), random width-16 rooms of every
height class (1..16 waves per grid: row slots past H idle, the 16-byte stop flags past 4 waves),
rooms with goals / lava / walls next to the key and the door (the KD and GOAL wave forms), an
all-absorbing interior (stops at its first sweep), max_sweeps caps, run_local + run_to
continuation, a fresh run_to (the k_target loop with |dV| on its last sweep only) and resume."""
import numpy as np
import pytest

import minigrid_dynamicprogramming_amd as mg
from minigrid_dynamicprogramming_amd.envs import DoorKeyEnv
from oracle import oracle

pytestmark = pytest.mark.gpu

EMPTY, WALL, FLOOR, DOOR, KEY, GOAL, LAVA = 1, 2, 3, 4, 5, 8, 9


def doorkey16(n, seed0=0):
    env = DoorKeyEnv(size=16)
    return np.stack([np.ascontiguousarray(env.generate(seed=seed0 + s)[0][..., 0].T) for s in range(n)]).astype(np.uint8)


def rooms16(H, n, seed, dense=False):
    """Width-16 rooms: closed border, a random interior, exactly one door and one key (the model's
    validation); `dense` puts goals / lava / walls around the key and the door."""
    rng = np.random.default_rng(seed)
    out = np.full((n, H, 16), WALL, np.uint8)
    for b in range(n):
        inner = rng.choice([EMPTY, WALL, FLOOR, GOAL, LAVA], size=(H - 2, 14), p=[0.66, 0.14, 0.06, 0.07, 0.07])
        out[b, 1:-1, 1:-1] = inner
        cells = [(y, x) for y in range(1, H - 1) for x in range(1, 15)]
        i, j = rng.choice(len(cells), 2, replace=False)
        (ky, kx), (dy, dx) = cells[i], cells[j]
        out[b, ky, kx] = KEY
        out[b, dy, dx] = DOOR
        if dense:
            for (y, x) in ((ky, kx), (dy, dx)):
                for (yy, xx) in ((y - 1, x), (y + 1, x), (y, x - 1), (y, x + 1)):
                    if 0 < yy < H - 1 and 0 < xx < 15 and out[b, yy, xx] not in (KEY, DOOR):
                        out[b, yy, xx] = rng.choice([EMPTY, GOAL, LAVA, WALL, FLOOR])
    return out


def solve(cells, dtype, rows, monkeypatch, **kw):
    monkeypatch.setenv("MGDP_DK_ROWS", rows)
    monkeypatch.setenv("MGDP_DK_HALF", "0")
    vi = mg.ValueIteration(cells, model="doorkey", dtype=dtype, **{k: v for k, v in kw.items() if k == "max_sweeps"})
    try:
        variant = vi.variant
        k = vi.solve()
        r = vi.result()
        return k, r.V, r.pi, variant
    finally:
        vi.close()


def check_vs_oracle(cells, dtype, monkeypatch, max_sweeps=10000):
    o = oracle.value_iteration(1, cells, dtype=dtype, max_sweeps=max_sweeps)
    k, V, pi, variant = solve(cells, dtype, "1", monkeypatch, max_sweeps=max_sweeps)
    assert variant == "dk_rows"
    assert k == o["sweeps"]
    np.testing.assert_array_equal(V, o["V"])
    np.testing.assert_array_equal(pi, o["pi"])
    return o


@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_doorkey16_reference_grids(dtype, monkeypatch):
    cells = doorkey16(96, seed0=7)
    check_vs_oracle(cells, dtype, monkeypatch)
    k0, V0, pi0, var0 = solve(cells, dtype, "0", monkeypatch)
    assert var0 == "dk_soa"
    k1, V1, pi1, _ = solve(cells, dtype, "1", monkeypatch)
    assert k0 == k1
    np.testing.assert_array_equal(V0, V1)
    np.testing.assert_array_equal(pi0, pi1)


# heights: 1 wave (3, 4 rows), 2 waves with idle row slots (5, 7), 4 (16), 5 (17, 20), 16 (64 rows)
@pytest.mark.parametrize("H", [3, 4, 5, 7, 16, 17, 20, 64])
def test_rooms_of_every_height(H, monkeypatch):
    cells = rooms16(H, 24, seed=H)
    check_vs_oracle(cells, "f32", monkeypatch)


@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_dense_key_door_goal_lava(dtype, monkeypatch):
    cells = rooms16(16, 48, seed=99, dense=True)
    check_vs_oracle(cells, dtype, monkeypatch)


def test_absorbing_interior_next_to_live_grids(monkeypatch):
    cells = doorkey16(8, seed0=300)
    dead = np.full((1, 16, 16), WALL, np.uint8)
    dead[0, 5, 5], dead[0, 9, 9] = KEY, DOOR  # nothing walkable: |dV| = 0 at its first sweep
    check_vs_oracle(np.concatenate([cells[:3], dead, cells[3:]]), "f32", monkeypatch)


@pytest.mark.parametrize("ms", [1, 2, 3, 17, 40])
def test_max_sweeps_caps(ms, monkeypatch):
    cells = doorkey16(12, seed0=500)
    o = check_vs_oracle(cells, "f32", monkeypatch, max_sweeps=ms)
    assert o["sweeps"] == ms


def test_protocol_continuation_and_fresh_run_to(monkeypatch):
    monkeypatch.setenv("MGDP_DK_ROWS", "1")
    monkeypatch.setenv("MGDP_DK_HALF", "0")
    cells = np.concatenate([doorkey16(10, seed0=900), rooms16(16, 6, seed=5, dense=True)])
    o = oracle.value_iteration(1, cells, dtype="f32")
    vi = mg.ValueIteration(cells, model="doorkey", dtype="f32")
    try:
        assert vi.variant == "dk_rows"
        vi.reset()
        k = vi.run_local()
        assert k == o["sweeps"]
        vi.run_to(k)
        vi.finish(k, 0.0)
        np.testing.assert_array_equal(vi.values(), o["V"])
        np.testing.assert_array_equal(vi.policy(), o["pi"])
        for first in (1, 5, 23):  # a fresh k_target loop to a fixed sweep, then on to K from HBM
            vi.reset()
            vi.run_to(first)
            dv = vi.run_to(k)
            vi.finish(k, dv)
            np.testing.assert_array_equal(vi.values(), o["V"])
            np.testing.assert_array_equal(vi.policy(), o["pi"])
        # every grid to exactly 7 sweeps: the literal loop capped at 7
        o7 = oracle.value_iteration(1, cells, dtype="f32", max_sweeps=7)
        vi.reset()
        vi.run_to(7)
        vi.finish(7, 0.0)
        np.testing.assert_array_equal(vi.values(), o7["V"])
        np.testing.assert_array_equal(vi.policy(), o7["pi"])
    finally:
        vi.close()


def test_resume_from_capped_checkpoint(monkeypatch):
    monkeypatch.setenv("MGDP_DK_ROWS", "1")
    monkeypatch.setenv("MGDP_DK_HALF", "0")
    cells = doorkey16(16, seed0=77)
    o = oracle.value_iteration(1, cells, dtype="f32")
    for cap in (1, 9, 30):
        capped = mg.ValueIteration(cells, model="doorkey", dtype="f32", max_sweeps=cap)
        try:
            capped.solve()
            ck = capped.checkpoint()
        finally:
            capped.close()
        vi = mg.ValueIteration(cells, model="doorkey", dtype="f32")
        try:
            assert vi.variant == "dk_rows"
            k = vi.resume(ck)
            assert k == o["sweeps"]
            r = vi.result()
            np.testing.assert_array_equal(r.V, o["V"])
            np.testing.assert_array_equal(r.pi, o["pi"])
        finally:
            vi.close()
