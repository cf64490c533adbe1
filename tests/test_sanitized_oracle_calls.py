"""Oracle entry points beyond the golden tables, for the sanitizer run (test_oracle_sanitized.py):
batched step with every action on grids of several families, finite-horizon / NoDeath VI, fp32
VI, and edge sizes.  Also a plain CPU test on its own (cheap)."""
import os

import numpy as np

import minigrid_dynamicprogramming_amd as mg
from oracle import oracle


def _cells(env_id, seeds):
    env = mg.make(env_id)
    return np.stack([np.ascontiguousarray(env.generate(seed=s)[0][..., 0].T) for s in seeds]).astype(np.uint8)


def test_vi_variants_run_clean():
    fr = _cells("MiniGrid-FourRooms-v0", range(3))
    dk = _cells("MiniGrid-DoorKey-8x8-v0", range(3))
    lava = _cells("MiniGrid-LavaCrossingS9N1-v0", range(3))
    for dtype in ("f32", "f64"):
        r = oracle.value_iteration(0, fr, dtype=dtype)
        assert r["converged"] if "converged" in r else True
        oracle.value_iteration(1, dk, dtype=dtype)
        oracle.value_iteration(0, lava, slip_p=0.9, dtype=dtype)
    # smallest grid the model takes (3x3: one free cell) and a max-size one
    tiny = np.full((1, 3, 3), 2, np.uint8)
    tiny[0, 1, 1] = 1
    oracle.value_iteration(0, tiny, dtype="f64")
    big = np.full((1, 32, 32), 2, np.uint8)
    big[0, 1:-1, 1:-1] = 1
    big[0, 30, 30] = 8
    oracle.value_iteration(0, big, dtype="f32")


def test_batched_env_steps_run_clean():
    for env_id in ("MiniGrid-DoorKey-8x8-v0", "MiniGrid-FourRooms-v0", "MiniGrid-LavaCrossingS9N1-v0"):
        env = mg.make(env_id)
        enc, agent = env.generate(seed=3)
        o = oracle.OracleEnv(enc, agent, env.max_steps, env.see_through_walls)
        rng = np.random.default_rng(0)
        for _ in range(200):
            img, r, term, trunc = o.step(int(rng.integers(0, 7)))
            assert img.shape == (env.agent_view_size, env.agent_view_size, 3)
            if term or trunc:
                o = oracle.OracleEnv(enc, agent, env.max_steps, env.see_through_walls)


def test_sanitizer_build_is_the_one_loaded_when_requested():
    want = os.environ.get("MGDP_ORACLE_LIB")
    if want:  # inside test_oracle_sanitized.py's child
        assert oracle.LIB_PATH == want and want.endswith("_asan.so")
        oracle.lib()
        with open("/proc/self/maps") as f:
            maps = f.read()
        assert want in maps and "libasan" in maps
