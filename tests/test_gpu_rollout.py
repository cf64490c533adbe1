"""Policy evaluation by rollout: execute the GPU value-iteration policy pi*
through the GPU step kernel from reset(seed) and check the discounted return of the surrogate
reward (R = 1 on entering the goal) equals V*[start].  For deterministic envs that return is
gamma^(n-1) for the n steps the rollout takes, computed here by the same repeated multiplication
the Bellman backups perform, so the check is exact (fp64).

This ties the two halves of the path together: the transition the DP models (csrc/vi.hip) and the
transition the env executes (csrc/envs.hip, bit-exact to reference step(), minigrid_env.py:520-590)
must agree on every state the optimal policy visits, including pickup/toggle in DoorKey.
"""
import numpy as np
import pytest

import minigrid_dynamicprogramming_amd as mg
from minigrid_dynamicprogramming_amd.core import OBJECT_TO_IDX
from minigrid_dynamicprogramming_amd.dp import state_index

pytestmark = pytest.mark.gpu

GAMMA = 0.99


def _gamma_pow(n):
    v = 1.0
    for _ in range(n - 1):
        v = GAMMA * v
    return v


@pytest.mark.parametrize("env_id,B", [
    ("MiniGrid-Empty-16x16-v0", 1),
    ("MiniGrid-Empty-Random-6x6-v0", 32),
    ("MiniGrid-FourRooms-v0", 64),
    ("MiniGrid-LavaCrossingS9N2-v0", 64),
    ("MiniGrid-LavaCrossingS11N5-v0", 64),
    ("MiniGrid-SimpleCrossingS11N5-v0", 64),
    ("MiniGrid-DoorKey-8x8-v0", 64),
    ("MiniGrid-DoorKey-16x16-v0", 32),
])
def test_optimal_policy_rollout_matches_value(env_id, B):
    venv = mg.MiniGridVecEnv(env_id, B)
    venv.reset(seed=0)
    st = venv.get_state()
    enc = st["enc"]
    model = "doorkey" if "DoorKey" in env_id else "xyd"
    res = mg.value_iteration(enc, model=model, gamma=GAMMA, tol=1e-6, dtype="f64")
    assert res.converged
    W = venv.W
    door = None
    if model == "doorkey":
        door = [tuple(np.argwhere(enc[b, :, :, 0] == OBJECT_TO_IDX["door"])[0]) for b in range(B)]

    def states(st):
        out = []
        for b in range(B):
            x, y, d = (int(v) for v in st["agent"][b])
            hk = dop = 0
            if model == "doorkey":
                hk = int(st["carry"][b, 0] == OBJECT_TO_IDX["key"])
                dx, dy = door[b]
                dop = int(st["enc"][b, dx, dy, 2] == 0)  # door state 0 = open (world_object.py:197-213)
            out.append((x, y, d, hk, dop))
        return out

    v_start = np.array([res.value(b, *states(st)[b]) for b in range(B)])
    done = np.zeros(B, bool)
    steps = np.zeros(B, np.int64)
    reached = np.zeros(B, bool)
    limit = 4 * venv.W * venv.H * (4 if model == "doorkey" else 1)
    for _ in range(limit):
        if done.all():
            break
        cur = states(st)
        acts = np.array([res.action(b, *cur[b]) if not done[b] else 6 for b in range(B)])
        assert (acts[~done] >= 0).all(), "policy queried on an absorbing state"
        _, rew, term, trunc, _ = venv.step(acts)
        live = ~done
        steps[live] += 1
        reached |= live & term & (rew > 0)
        done |= live & (term | trunc)
        st = venv.get_state()
    venv.close()
    solvable = v_start > 0
    assert solvable.any()
    assert (reached == solvable).all(), (env_id, np.flatnonzero(reached != solvable))
    for b in np.flatnonzero(solvable):
        assert v_start[b] == _gamma_pow(int(steps[b])), (env_id, b, int(steps[b]), v_start[b])
