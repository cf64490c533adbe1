"""Box(contains=...) on the HIP step (csrc/envs.hip contents plane, mgdp_envs_set_contents; reference
minigrid/core/world_object.py:272-294 and minigrid_env.py:556-575): toggling a Box puts what it holds
in its cell, a carried Box keeps it, drop puts it back.  Pinned to the reference's own rollouts
(tests/golden/traj_box.npz, make_golden_box.py) and, at batch scale, to the oracle's orc_step_held."""
import hashlib

import numpy as np
import pytest

import minigrid_dynamicprogramming_amd as mg
from minigrid_dynamicprogramming_amd.core import Ball, Box, Key
from minigrid_dynamicprogramming_amd.vector import MiniGridVecEnv
from oracle import oracle
from tests.golden_util import load

pytestmark = pytest.mark.gpu


def digest(a):
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest()[:8], dtype=np.uint64)[0]


@pytest.mark.parametrize("group", ["8", "4", "2", "1"])
def test_box_trajectories_match_reference(group, monkeypatch):
    monkeypatch.setenv("MGDP_STEP_GROUP", group)
    t = load("traj_box.npz")
    B = t["actions"].shape[0]
    venv = MiniGridVecEnv("MiniGrid-Empty-8x8-v0", B)  # an 8x8 handle; the grids are the fixture's
    venv.load(t["init_enc"], t["init_agent"], max_steps=t["max_steps"], see_through=[False] * B, held=t["init_held"])
    np.testing.assert_array_equal(venv.observe()["image"], t["init_image"])
    for i in range(t["actions"].shape[1]):
        obs, rew, term, trunc, _ = venv.step(t["actions"][:, i])
        ctx = f"box step {i}"
        np.testing.assert_array_equal(obs["image"], t["image"][:, i], err_msg=ctx)
        np.testing.assert_array_equal(obs["direction"], t["direction"][:, i], err_msg=ctx)
        np.testing.assert_array_equal(rew, t["reward"][:, i], err_msg=ctx)
        np.testing.assert_array_equal(term, t["terminated"][:, i].astype(bool), err_msg=ctx)
        np.testing.assert_array_equal(trunc, t["truncated"][:, i].astype(bool), err_msg=ctx)
        st = venv.get_state()
        np.testing.assert_array_equal(st["agent"], t["agent"][:, i], err_msg=ctx)
        np.testing.assert_array_equal(st["carry"], t["carry"][:, i], err_msg=ctx)
        np.testing.assert_array_equal(st["carry_held"], t["carry_held"][:, i], err_msg=ctx)
        for b in range(B):
            assert digest(st["enc"][b]) == t["grid_digest"][b, i], ctx
            assert digest(st["held"][b]) == t["held_digest"][b, i], ctx
    st = venv.get_state()
    np.testing.assert_array_equal(st["enc"], t["final_enc"])
    np.testing.assert_array_equal(st["held"], t["final_held"])
    venv.close()


def random_box_rooms(B, W, seed):
    """B walled W x W rooms with boxes (holding a key, a ball, an empty box or nothing), a few keys
    and balls, and an agent on a free cell -- the oracle's and the kernel's common input."""
    rng = np.random.default_rng(seed)
    enc = np.zeros((B, W, W, 3), np.uint8)
    enc[..., 0] = 1
    enc[:, 0, :, 0] = enc[:, -1, :, 0] = enc[:, :, 0, 0] = enc[:, :, -1, 0] = 2
    enc[:, 0, :, 1] = enc[:, -1, :, 1] = enc[:, :, 0, 1] = enc[:, :, -1, 1] = 5
    held = np.zeros_like(enc)
    agent = np.zeros((B, 3), np.int32)
    inner = [(x, y) for x in range(1, W - 1) for y in range(1, W - 1)]
    for b in range(B):
        cells = rng.permutation(len(inner))
        for n, ci in enumerate(cells[: len(inner) // 2]):
            x, y = inner[ci]
            kind = rng.integers(0, 6)
            if kind < 4:
                enc[b, x, y] = (7, rng.integers(0, 6), 0)
                h = rng.integers(0, 4)
                if h:
                    held[b, x, y] = ((5, 6, 7)[h - 1], rng.integers(0, 6), 0)
            else:
                enc[b, x, y] = ((5, 6)[kind - 4], rng.integers(0, 6), 0)
        x, y = inner[cells[-1]]
        agent[b] = (x, y, rng.integers(0, 4))
    return enc, agent, held


@pytest.mark.parametrize("group", ["2", "8"])
def test_box_rooms_random_actions_vs_oracle(group, monkeypatch):
    """4101 crowded box rooms, 128 steps of pickup / drop / toggle-heavy random actions: every obs
    byte, reward, flag, agent, carry, carried contents and the final grids and contents equal the
    oracle's orc_step_batch_held."""
    monkeypatch.setenv("MGDP_STEP_GROUP", group)
    B, W, steps = 4101, 8, 128
    enc, agent, held = random_box_rooms(B, W, seed=11)
    venv = MiniGridVecEnv("MiniGrid-Empty-8x8-v0", B)
    venv.load(enc, agent, max_steps=[1000] * B, see_through=[False] * B, held=held)
    ob = oracle.OracleBatch(enc, agent, 1000, False, held=held)
    rng = np.random.default_rng(5)
    p = np.array([0.12, 0.12, 0.2, 0.2, 0.16, 0.16, 0.04])
    for t in range(steps):
        a = rng.choice(7, size=B, p=p).astype(np.int32)
        obs, rew, term, trunc, _ = venv.step(a)
        ob.step(a)
        np.testing.assert_array_equal(obs["image"], ob.obs, err_msg=f"step {t}")
        np.testing.assert_array_equal(rew, ob.reward, err_msg=f"step {t}")
        np.testing.assert_array_equal(term, ob.terminated.astype(bool))
    st = venv.get_state()
    np.testing.assert_array_equal(st["agent"], ob.state[:, :3])
    np.testing.assert_array_equal(st["carry"], ob.carry)
    np.testing.assert_array_equal(st["carry_held"], ob.held_carry)
    np.testing.assert_array_equal(st["held"], ob.held_encoding())
    enc_o = np.stack([q[:, : W * W].reshape(B, W, W).transpose(0, 2, 1) for q in (ob.ty, ob.co, ob.st)], axis=-1)
    np.testing.assert_array_equal(st["enc"], enc_o)
    opened = (enc[..., 0] == 7).sum() - (st["enc"][..., 0] == 7).sum()
    assert opened > 0 and (st["carry_held"][:, 0] > 0).any()  # the paths were exercised
    venv.close()


def test_single_env_box_contents_api():
    """The gymnasium surface: a Box(contains=Key) set on env.grid opens to the key; a carried Box
    keeps its Ball (env.carrying.contains) and returns it to the grid on drop."""
    env = mg.make("MiniGrid-Empty-8x8-v0")
    env.reset(seed=0)
    x, y = env.agent_pos
    env.agent_dir = 0  # facing east
    env.grid.set(x + 1, y, Box("red", contains=Key("blue")))
    obs, *_ = env.step(mg.Actions.toggle)
    k = env.grid.get(x + 1, y)
    assert k is not None and k.type == "key" and k.color == "blue"
    assert tuple(obs["image"][3, 5]) == (5, 2, 0)  # the key right in front of the agent
    env.grid.set(x + 1, y, Box("green", contains=Ball("purple")))
    env.step(mg.Actions.pickup)
    assert env.carrying.type == "box" and env.carrying.contains is not None
    assert env.carrying.contains.type == "ball" and env.carrying.contains.color == "purple"
    assert env.grid.get(x + 1, y) is None
    env.step(mg.Actions.drop)
    b = env.grid.get(x + 1, y)
    assert env.carrying is None and b.type == "box" and b.contains.type == "ball"
    env.step(mg.Actions.toggle)
    assert env.grid.get(x + 1, y).type == "ball"
    env.close()


def test_contents_are_validated():
    venv = MiniGridVecEnv("MiniGrid-Empty-5x5-v0", 2)
    venv.reset(seed=0)
    held = np.zeros((2, 5, 5, 3), np.uint8)
    held[0, 2, 2] = (5, 1, 0)  # a key "held" by a cell that is no Box
    with pytest.raises(ValueError):  # MGDP_E_INVALID
        venv.set_contents(held)
    st = venv.get_state()
    enc = st["enc"].copy()
    enc[0, 2, 2] = (7, 0, 0)
    venv.load(enc, st["agent"])
    venv.set_contents(held)  # now it sits on a Box
    h, ch = venv.get_contents()
    assert tuple(h[0, 2, 2]) == (5, 1, 0) and not ch.any()
    venv.load(enc, st["agent"])  # a load clears the contents of the loaded envs
    assert not venv.get_contents()[0].any()
    carry = np.array([[7, 3], [0, 0]], np.int32)  # env 0 carries a purple Box
    venv.L.mgdp_envs_set_state(venv.h, None, carry.ctypes.data, None, None)
    with pytest.raises(ValueError):  # env 1 carries nothing: it cannot hold contents
        venv.set_contents(carry_held=np.array([[5, 1, 0], [6, 2, 0]], np.int32))
    venv.set_contents(carry_held=np.array([[5, 1, 0], [0, 0, 0]], np.int32))
    assert tuple(venv.get_contents()[1][0]) == (5, 1, 0)
    venv.L.mgdp_envs_set_state(venv.h, None, carry.ctypes.data, None, None)  # a new carry holds nothing
    assert not venv.get_contents()[1].any()
    venv.close()


def test_masked_load_replaces_only_masked_envs():
    """mgdp_envs_load with a mask (auto-reset of some envs; one staging copy + a scatter kernel):
    the masked envs get the new grids, agents, max_steps, see_through, a cleared carry and no Box
    contents; every other env keeps its state and contents byte for byte."""
    B, W = 4096 + 5, 8
    enc0, agent0, held0 = random_box_rooms(B, W, seed=11)
    enc1, agent1, _ = random_box_rooms(B, W, seed=12)
    venv = MiniGridVecEnv("MiniGrid-Empty-8x8-v0", B)
    ms0 = np.full(B, 77, np.int32)
    venv.load(enc0, agent0, max_steps=ms0, see_through=[False] * B, held=held0)
    rng = np.random.default_rng(5)
    for _ in range(7):  # move agents / carry things, so the kept envs' state is not the loaded one
        venv.step(rng.integers(0, 7, B).astype(np.int32))
    before = venv.get_state()
    mask = (rng.random(B) < 0.3).astype(np.uint8)
    ms1 = np.full(B, 55, np.int32)
    venv.load(enc1, agent1, max_steps=ms1, see_through=[True] * B, mask=mask)
    after = venv.get_state()
    m = mask.astype(bool)
    np.testing.assert_array_equal(after["enc"][m], enc1[m])
    np.testing.assert_array_equal(after["agent"][m], agent1[m])
    assert (after["carry"][m] == 0).all() and (after["step_count"][m] == 0).all()
    assert (after["held"][m] == 0).all() and (after["carry_held"][m] == 0).all()
    for k in ("enc", "agent", "carry", "step_count", "held", "carry_held"):
        np.testing.assert_array_equal(after[k][~m], before[k][~m], err_msg=k)
    # the masked envs step with their new max_steps / see_through: compare with a fresh handle
    ref = MiniGridVecEnv("MiniGrid-Empty-8x8-v0", int(m.sum()))
    ref.load(enc1[m], agent1[m], max_steps=ms1[m], see_through=[True] * int(m.sum()))
    a = rng.integers(0, 7, B).astype(np.int32)
    obs, rew, term, trunc, _ = venv.step(a)
    robs, rrew, rterm, rtrunc, _ = ref.step(a[m])
    np.testing.assert_array_equal(obs["image"][m], robs["image"])
    np.testing.assert_array_equal(rew[m], rrew)
    ref.close()
    venv.close()
