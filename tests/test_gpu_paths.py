"""Solver paths selected by handle-creation knobs (read from the environment by mgdp_vi_create),
each against the oracle: the chained batched solve (run_local -> run_to with K in device memory)
and the two-wait form (MGDP_CHAIN=0); a lone grid launched per solve (MGDP_PERSISTENT=0) through
the chain; the batched XYD path without the one-wave solver (MGDP_WAVE2=0, two cells per thread);
and the separate reduce kernel against the in-kernel reduction (MGDP_INKERNEL_MAX)."""
import os

import numpy as np
import pytest

import minigrid_dynamicprogramming_amd as mg
from oracle import oracle
from tests.golden_util import cells_from_enc, load

pytestmark = pytest.mark.gpu


def random_grids(n, W, H, seed):
    rng = np.random.default_rng(seed)
    out = np.full((n, H, W), 2, np.uint8)
    for i in range(n):
        out[i, 1:-1, 1:-1] = rng.choice(np.array([1, 1, 1, 1, 2, 9], np.uint8), size=(H - 2, W - 2))
        out[i, rng.integers(1, H - 1), rng.integers(1, W - 1)] = 8
    return out


def solve_with(env, cells, model_id, dtype, **kw):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        r = mg.value_iteration(cells, model="xyd" if model_id == 0 else "doorkey", dtype=dtype, **kw)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    o = oracle.value_iteration(model_id, cells, dtype=dtype, slip_p=kw.get("slip_p"))
    assert r.sweeps == o["sweeps"]
    np.testing.assert_array_equal(r.pi, o["pi"])
    np.testing.assert_array_equal(r.V, o["V"])
    return r


@pytest.mark.parametrize("env", [{"MGDP_CHAIN": "0"}, {"MGDP_CHAIN": "1"}, {"MGDP_WAVE2": "0"},
                                 {"MGDP_INKERNEL_MAX": "0"}, {"MGDP_INKERNEL_MAX": "100000"}])
@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_batched_xyd_paths(env, dtype):
    solve_with(env, random_grids(40, 13, 11, seed=3), 0, dtype)


@pytest.mark.parametrize("env", [{"MGDP_CHAIN": "0"}, {"MGDP_CHAIN": "1"}])
def test_batched_doorkey_and_slip_paths(env):
    dk = mg.make("MiniGrid-DoorKey-8x8-v0")
    cells = np.stack([np.ascontiguousarray(dk.generate(seed=s)[0][..., 0].T) for s in range(20)]).astype(np.uint8)
    solve_with(env, cells, 1, "f32")
    solve_with(env, random_grids(20, 9, 9, seed=4), 0, "f64", slip_p=0.9)


@pytest.mark.parametrize("name", ["empty16_s0", "fourrooms_s1", "doorkey16_s0"])
def test_lone_grid_launch_per_solve(name):
    t = load(f"table_{name}.npz")
    solve_with({"MGDP_PERSISTENT": "0"}, cells_from_enc(t["enc"]), int(t["model"]), "f32")
