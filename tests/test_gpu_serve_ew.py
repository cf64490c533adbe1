"""The served lone deterministic XYD grid on fused_serve_xyd (east / west fronts by DPP, two LDS
planes, three rotating register sets; csrc/vi_loops.h) against the CPU oracle, bit for bit: sweeps,
V, pi and the last sweep's dV.  Covers grids whose wave edges allow the DPP path and grids whose
first / last lane of a wave has a valid neighbour in the next wave (the in-kernel fallback to
fused_fast_xyd_soa), both in one resident server through new-grid requests, and the host switch
MGDP_SERVE_EW=0.  Round 6: every case also on the two-sweeps-per-barrier loop (fused_serve_pair, the
default; MGDP_SERVE_PAIR=0 keeps fused_serve_xyd), including odd and even max_sweeps caps (a pair may
compute past the cap) and wide grids (W up to 50: neighbours two rows away read from the pads)."""
import numpy as np
import pytest

import minigrid_dynamicprogramming_amd as mg
from oracle import oracle

pytestmark = pytest.mark.gpu

EMPTY, WALL, GOAL, LAVA = 1, 2, 8, 9


def random_grid(rng, W, H, p_wall=0.15, p_lava=0.07):
    g = np.full((H, W), EMPTY, np.uint8)
    g[0, :] = g[-1, :] = WALL
    g[:, 0] = g[:, -1] = WALL
    inner = rng.random((H - 2, W - 2))
    g[1:-1, 1:-1][inner < p_wall] = WALL
    g[1:-1, 1:-1][(inner >= p_wall) & (inner < p_wall + p_lava)] = LAVA
    y, x = rng.integers(1, H - 1), rng.integers(1, W - 1)
    g[y, x] = GOAL
    return g


def wave_edge_open(g):
    """True if some wave's first / last cell and its neighbour across the wave boundary are both
    walkable (the grid then takes the fused_fast_xyd_soa fallback inside the server)."""
    flat = g.reshape(-1)
    free = (flat == EMPTY)
    for c in range(63, flat.size - 1, 64):
        if free[c] and free[c + 1]:
            return True
    return False


def solve_served(vi):
    vi.solve()
    return vi.sweeps, vi.dv, vi.values(), vi.policy()


def check(g, res, dtype):
    o = oracle.value_iteration(0, g[None], dtype=dtype)
    k, dv, V, pi = res
    assert k == o["sweeps"]
    assert dv == o["dv"]
    np.testing.assert_array_equal(V, o["V"])
    np.testing.assert_array_equal(pi, o["pi"])


PAIR = pytest.mark.parametrize("pair", ["0", "1"])


def expected_variant(W, pair):
    return "serve_pair" if pair == "1" else "serve_ew"


@PAIR
@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_served_ew_random_grids(dtype, pair, monkeypatch):
    monkeypatch.setenv("MGDP_PERSISTENT", "1")
    monkeypatch.setenv("MGDP_SERVE_PAIR", pair)
    rng = np.random.default_rng(7)
    seen_open = seen_closed = 0
    for i in range(32):
        while True:
            if i % 4 == 3:  # wide grids: widths 17..50
                W, H = int(rng.integers(17, 51)), int(rng.integers(3, 8))
            else:
                W, H = int(rng.integers(5, 17)), int(rng.integers(5, 17))
            if 64 < W * H <= 256:
                break
        g = random_grid(rng, W, H)
        if wave_edge_open(g):
            seen_open += 1
        else:
            seen_closed += 1
        vi = mg.ValueIteration(g[None], dtype=dtype)
        assert vi.persistent
        assert vi.variant == expected_variant(W, pair), (W, vi.variant)
        check(g, solve_served(vi), dtype)
        check(g, solve_served(vi), dtype)  # a second request on the resident server
        vi.close()
    assert seen_open and seen_closed


@PAIR
def test_served_ew_grid_changes_between_requests(pair, monkeypatch):
    """One resident server, new grids handed over between requests, alternating between grids the
    DPP path takes and grids that fall back (serve_ew_ok is re-evaluated per grid)."""
    monkeypatch.setenv("MGDP_PERSISTENT", "1")
    monkeypatch.setenv("MGDP_SERVE_PAIR", pair)
    rng = np.random.default_rng(11)
    W, H = 10, 10
    grids = []
    while len(grids) < 6:
        g = random_grid(rng, W, H, p_wall=0.1, p_lava=0.05)
        if wave_edge_open(g) == (len(grids) % 2 == 1):
            grids.append(g)
    vi = mg.ValueIteration(grids[0][None], dtype="f32")
    for g in grids:
        vi.load(g[None])
        check(g, solve_served(vi), "f32")
    vi.close()


@pytest.mark.parametrize("ew,pair", [("0", "1"), ("1", "0"), ("1", "1")])
def test_served_empty16(ew, pair, monkeypatch):
    """The headline grid on every host setting: 29 sweeps, bit-exact."""
    monkeypatch.setenv("MGDP_PERSISTENT", "1")
    monkeypatch.setenv("MGDP_SERVE_EW", ew)
    monkeypatch.setenv("MGDP_SERVE_PAIR", pair)
    enc, _ = mg.make("MiniGrid-Empty-16x16-v0").generate(seed=0)
    g = np.ascontiguousarray(enc[:, :, 0].T)
    vi = mg.ValueIteration(g[None], dtype="f32")
    assert vi.variant == ("serve_pair" if ew == "1" and pair == "1" else ("serve_ew" if ew == "1" else vi.variant))
    for _ in range(3):
        res = solve_served(vi)
        assert res[0] == 29
        check(g, res, "f32")
    vi.close()


@PAIR
def test_served_ew_max_sweeps_cap(pair, monkeypatch):
    """Stopped by max_sweeps instead of the rule: V_k and the pi of sweep k as the oracle's (every
    cap 1..13: both halves of a pair, both loop positions' parities; and caps past the rule's K)."""
    monkeypatch.setenv("MGDP_PERSISTENT", "1")
    monkeypatch.setenv("MGDP_SERVE_PAIR", pair)
    enc, _ = mg.make("MiniGrid-Empty-16x16-v0").generate(seed=0)
    g = np.ascontiguousarray(enc[:, :, 0].T)
    for cap in list(range(1, 14)) + [28, 29, 30]:
        vi = mg.ValueIteration(g[None], dtype="f32", max_sweeps=cap)
        k, dv, V, pi = solve_served(vi)
        o = oracle.value_iteration(0, g[None], dtype="f32", max_sweeps=cap)
        assert k == o["sweeps"] == min(cap, 29)
        assert dv == o["dv"]
        np.testing.assert_array_equal(V, o["V"])
        np.testing.assert_array_equal(pi, o["pi"])
        vi.close()
