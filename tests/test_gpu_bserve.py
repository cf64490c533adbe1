"""The resident batch server (csrc/vi_kernels.h vi_bserve_kernel): a one-wave
deterministic XYD batch within the server's resident capacity stays on the device between solves
and a solve is a request word.  Every request must be a full solve from V_0 = 0 (nothing carried
over): each case solves several times on one resident launch and checks sweeps, dV, V, pi and the
executed sweeps against the oracle's global loop after every solve, with new grids (a new launch)
between requests, the capped rule, solve_last, the server off (MGDP_BSERVE=0) and timing on (a
timed solve is a launch) giving the same bits."""
import os

import numpy as np
import pytest

import minigrid_dynamicprogramming_amd as mg
from minigrid_dynamicprogramming_amd import gen
from oracle import oracle
from tests.test_gpu_wave2 import random_grids

pytestmark = pytest.mark.gpu


def _handle(cells, dtype, env=None, **kw):
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        return mg.ValueIteration(cells, dtype=dtype, **kw)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _check(vi, o, k):
    assert k == o["sweeps"]
    np.testing.assert_array_equal(vi.values(), o["V"])
    np.testing.assert_array_equal(vi.policy(), o["pi"])
    np.testing.assert_array_equal(vi.grid_sweeps(), o["grid_sweeps"])


CASES = [("MiniGrid-FourRooms-v0", 512, "f32"), ("MiniGrid-LavaCrossingS11N5-v0", 2048, "f32"),
         ("MiniGrid-Empty-16x16-v0", 300, "f64"), ("MiniGrid-LavaCrossingS9N1-v0", 1000, "f64")]


@pytest.mark.parametrize("env_id,B,dtype", CASES)
def test_served_batch_solves_are_fresh_and_exact(env_id, B, dtype):
    cells = gen.generate(env_id, 0, B, enc=False, cells=True, agent=False)["cells"]
    o = oracle.value_iteration(0, cells, dtype=dtype, nthreads=16, fixed_point=True)
    vi = _handle(cells, dtype)
    try:
        n = 6
        ks = [vi.solve() for _ in range(n)]  # one resident launch serves these (no result read between)
        assert ks == [o["sweeps"]] * n
        assert vi.dv == o["dv"]
        clk = vi.serve_clock()  # stops the server: its solve count comes with its exit word
        assert clk["launches"] >= 1 and clk["solves"] >= n - 1, clk
        _check(vi, o, ks[-1])
        # a result read stops the server; the next solve relaunches it: still exact
        k = vi.solve()
        _check(vi, o, k)
        # new grids: a new launch on the new cells, several requests again
        other = gen.generate(env_id, 1000, B, enc=False, cells=True, agent=False)["cells"]
        o2 = oracle.value_iteration(0, other, dtype=dtype, nthreads=16, fixed_point=True)
        vi.load(other)
        for _ in range(3):
            k = vi.solve()
            assert k == o2["sweeps"]
        _check(vi, o2, k)
        vi.load(cells)
        k = vi.solve()
        _check(vi, o, k)
    finally:
        vi.close()


@pytest.mark.parametrize("W,H,goals", [(9, 7, 2), (13, 13, 1), (19, 19, 1), (21, 21, 3)])
def test_served_random_batches(W, H, goals):
    cells = random_grids(777, W, H, seed=W * H, goals=goals)
    o = oracle.value_iteration(0, cells, dtype="f32", nthreads=16, fixed_point=True)
    vi = _handle(cells, "f32")
    try:
        for _ in range(4):
            k = vi.solve()
            assert k == o["sweeps"]
        assert vi.serve_clock()["solves"] >= 3
        _check(vi, o, k)
    finally:
        vi.close()


def test_server_off_and_timed_solves_give_the_same_bits():
    cells = gen.generate("MiniGrid-FourRooms-v0", 7, 1024, enc=False, cells=True, agent=False)["cells"]
    o = oracle.value_iteration(0, cells, dtype="f32", nthreads=16, fixed_point=True)
    served = _handle(cells, "f32")
    off = _handle(cells, "f32", {"MGDP_BSERVE": "0"})
    try:
        for h in (served, off):
            for _ in range(3):
                k = h.solve()
            _check(h, o, k)
        served.enable_timing(True)  # a timed solve is a launch of the fused kernel
        for _ in range(2):
            k = served.solve()
        _, launches = served.kernel_time()
        assert launches == 2
        _check(served, o, k)
        served.enable_timing(False)
        served.solve()
        served.solve()
        assert served.serve_clock()["solves"] >= 1
        off.solve()
        assert off.serve_clock()["solves"] == 0
    finally:
        served.close()
        off.close()


@pytest.mark.parametrize("cap", [1, 2, 5, 17])
def test_served_capped_batches(cap):
    """max_sweeps below the grids' own stopping sweeps: the served request reports K = cap with some
    grids unfinished (dV > 0); the solve continues on the general path (run_to) and must equal the
    oracle's capped loop, request after request."""
    cells = random_grids(400, 16, 16, seed=11, goals=1)
    o = oracle.value_iteration(0, cells, dtype="f32", nthreads=16, max_sweeps=cap)
    vi = _handle(cells, "f32", max_sweeps=cap)
    try:
        for _ in range(3):
            assert vi.solve() == o["sweeps"] == cap
            assert not vi.converged
        np.testing.assert_array_equal(vi.values(), o["V"])
        np.testing.assert_array_equal(vi.policy(), o["pi"])
    finally:
        vi.close()


def test_solve_last_and_synchronize():
    cells = gen.generate("MiniGrid-LavaCrossingS11N5-v0", 3, 4096, enc=False, cells=True, agent=False)["cells"]
    o = oracle.value_iteration(0, cells, dtype="f32", nthreads=16, fixed_point=True)
    vi = _handle(cells, "f32")
    try:
        for _ in range(3):
            vi.solve()
        k = vi.solve(True)  # the request tells the server to leave after it
        vi.synchronize()
        _check(vi, o, k)
        for _ in range(2):
            vi.solve()
        vi.synchronize()  # waits for the exit word of a resident server told to quit
        _check(vi, o, vi.sweeps)
    finally:
        vi.close()


def test_protocol_run_local_does_not_start_a_batch_server():
    """A caller driving run_local / run_to itself (the sharded protocols) gets launches: a resident
    batch server would hold the CU slots a collective between them needs."""
    cells = random_grids(256, 11, 11, seed=5, goals=1)
    o = oracle.value_iteration(0, cells, dtype="f32", nthreads=16, fixed_point=True)
    vi = _handle(cells, "f32")
    try:
        vi.reset()
        K = vi.run_local()
        dv = vi.run_to(K)
        vi.finish(K, dv)
        assert K == o["sweeps"]
        assert vi.serve_clock()["solves"] == 0
        np.testing.assert_array_equal(vi.values(), o["V"])
        np.testing.assert_array_equal(vi.policy(), o["pi"])
        assert vi.solve() == o["sweeps"] and vi.solve() == o["sweeps"]  # solve() itself is served
        assert vi.serve_clock()["solves"] >= 1
    finally:
        vi.close()


@pytest.mark.parametrize("B", [2, 3, 64])
def test_small_served_batches(B):
    cells = random_grids(B, 13, 13, seed=B, goals=1)
    o = oracle.value_iteration(0, cells, dtype="f64", nthreads=4, fixed_point=True)
    vi = _handle(cells, "f64")
    try:
        for _ in range(3):
            assert vi.solve() == o["sweeps"]
        _check(vi, o, o["sweeps"])
    finally:
        vi.close()


@pytest.mark.parametrize("extra", [1, 777])
def test_multi_grid_server_past_capacity(extra):
    """MGDP_BSERVE=2: a batch past the server's resident capacity, several grids per workgroup (the
    multi-grid loop).  Also the regression test of the write-through exit store's data hazard (an asm
    global_store_dwordx4 without its s_nop: the loop's next VALU overwrote the store's first data
    register before it was read, and some 4-lane groups stored a stale first dword -- ~0.3 % of the
    grids wrong here before the fix)."""
    import torch

    cap = 32 * torch.cuda.get_device_properties(0).multi_processor_count  # 9x7 grids: 8 waves per SIMD
    cells = random_grids(cap + extra, 9, 7, seed=extra, goals=2)
    o = oracle.value_iteration(0, cells, dtype="f32", nthreads=16, fixed_point=True)
    vi = _handle(cells, "f32", {"MGDP_BSERVE": "2"})
    try:
        for _ in range(3):
            assert vi.solve() == o["sweeps"]
        assert vi.serve_clock()["solves"] >= 2
        _check(vi, o, o["sweeps"])
    finally:
        vi.close()
