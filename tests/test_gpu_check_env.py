"""gymnasium's env checker, restated, on every registered id (the reference's tests/test_envs.py:30-36
runs `gymnasium.utils.env_checker.check_env(env)` on each of its ids).

gymnasium is a third-party dependency of the reference (pyproject.toml:29, "gymnasium>=0.28.1")
that is not importable in this image, so the checker itself cannot run; this file restates the
checks its published check_env performs on an Env with no render mode (gymnasium 0.28 / 0.29 / 1.0
`gymnasium/utils/env_checker.py`): the spaces are Spaces; reset() returns (obs, info dict) with obs
in the observation space; reset takes `seed` and `options` keywords; reset(seed=123) twice gives
equal observations and leaves np_random in the same state, reset(seed=456) a different one;
reset(options={}) works; step() returns a 5-tuple (obs in the space, a finite int / float reward,
bool terminated / truncated, info dict); the same seed and action give the same step (1.0's
check_step_determinism); render metadata is well-formed.  Parity unpinned (no reference output
exists for the checker here): these are the checker's assertions, not recorded values."""
import copy
import inspect
import math

import numpy as np
import pytest

from minigrid_dynamicprogramming_amd._gym import Env, spaces
from minigrid_dynamicprogramming_amd.registry import registry

pytestmark = pytest.mark.gpu

SPECS = sorted(registry.values(), key=lambda s: s.id)


def data_equivalence(a, b) -> bool:
    """gymnasium.utils.env_checker.data_equivalence: same type, same keys / items, equal arrays of
    equal dtype."""
    if type(a) is not type(b):
        return False
    if isinstance(a, dict):
        return a.keys() == b.keys() and all(data_equivalence(a[k], b[k]) for k in a)
    if isinstance(a, (tuple, list)):
        return len(a) == len(b) and all(data_equivalence(x, y) for x, y in zip(a, b))
    if isinstance(a, np.ndarray):
        return a.shape == b.shape and a.dtype == b.dtype and bool(np.all(a == b))
    return a == b


def obs_in_space(env, obs):
    sp = env.observation_space
    assert isinstance(obs, dict) and sp.contains(obs), "observation not in the observation space"
    img = obs["image"]
    assert isinstance(img, np.ndarray) and img.dtype == np.dtype(sp["image"].dtype)  # Box dtype check


@pytest.mark.parametrize("spec", SPECS, ids=[s.id for s in SPECS])
def test_check_env_restated(spec):
    env = spec.make()
    assert isinstance(env, Env)
    assert isinstance(env.action_space, spaces.Space)
    assert isinstance(env.observation_space, spaces.Space)
    # render metadata (check_env's render checks, render_mode None)
    assert isinstance(env.metadata.get("render_modes"), list)
    assert isinstance(env.metadata.get("render_fps"), int)
    # reset: return type
    res = env.reset(seed=0)
    assert isinstance(res, tuple) and len(res) == 2
    obs, info = res
    obs_in_space(env, obs)
    assert isinstance(info, dict)
    # reset: seed and options keywords
    params = inspect.signature(env.reset).parameters
    assert "seed" in params and "options" in params
    # reset: seeding
    obs_1, _ = env.reset(seed=123)
    obs_in_space(env, obs_1)
    assert env.unwrapped._np_random is not None
    seed_123_rng = copy.deepcopy(env.unwrapped._np_random)
    obs_2, _ = env.reset(seed=123)
    obs_in_space(env, obs_2)
    assert data_equivalence(obs_1, obs_2)
    assert env.unwrapped._np_random.bit_generator.state == seed_123_rng.bit_generator.state
    obs_3, _ = env.reset(seed=456)
    obs_in_space(env, obs_3)
    assert env.unwrapped._np_random.bit_generator.state != seed_123_rng.bit_generator.state
    # reset: options
    obs_4, _ = env.reset(options={})
    obs_in_space(env, obs_4)
    # step: return types
    env.reset(seed=0)
    action = env.action_space.sample()
    assert env.action_space.contains(action)
    res = env.step(action)
    assert isinstance(res, tuple) and len(res) == 5
    obs, reward, terminated, truncated, info = res
    obs_in_space(env, obs)
    assert isinstance(reward, (int, float, np.integer, np.floating)) and math.isfinite(float(reward))
    assert isinstance(terminated, (bool, np.bool_)) and isinstance(truncated, (bool, np.bool_))
    assert isinstance(info, dict)
    # step determinism (check_step_determinism): same seed, same action -> same step
    env.action_space.seed(123)
    a = env.action_space.sample()
    env.reset(seed=123)
    r0 = env.step(a)
    env.reset(seed=123)
    r1 = env.step(a)
    assert data_equivalence(r0[0], r1[0]) and r0[1:] == r1[1:]
    env.close()
