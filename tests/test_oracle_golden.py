"""Pin the CPU oracle (oracle/) to golden vectors captured from the reference itself.

Transition tables were extracted by driving the reference MiniGridEnv.step()
(minigrid/minigrid_env.py:520-590) from every enumerated state; trajectories are 256-step rollouts
of the reference env; V*/pi*/sweeps come from an independent numpy Jacobi over those tables.
"""
import ctypes

import numpy as np
import pytest

from oracle import oracle
from tests.golden_util import SEE_THROUGH, cells_from_enc, load, table_names, traj_names


@pytest.mark.parametrize("name", table_names())
def test_transition_table_matches_reference(name):
    t = load(f"table_{name}.npz")
    model = int(t["model"])
    nxt, rew, done = oracle.build_table(model, cells_from_enc(t["enc"]))
    np.testing.assert_array_equal(nxt, t["nxt"])
    np.testing.assert_array_equal(done, t["done"])
    np.testing.assert_array_equal(rew, t["rew"])


@pytest.mark.parametrize("name", table_names())
def test_vi_fp64_matches_golden(name):
    t = load(f"table_{name}.npz")
    model = int(t["model"])
    res = oracle.value_iteration(model, cells_from_enc(t["enc"]), 0.99, 1e-6, dtype="f64")
    assert res["sweeps"] == int(t["sweeps"])
    np.testing.assert_array_equal(res["pi"][0], t["pi"])
    np.testing.assert_allclose(res["V"][0], t["V"], rtol=0, atol=1e-12)
    if model == 0:
        rs = oracle.value_iteration(model, cells_from_enc(t["enc"]), 0.99, 1e-6, slip_p=0.9, dtype="f64")
        assert rs["sweeps"] == int(t["sweeps_slip"])
        np.testing.assert_array_equal(rs["pi"][0], t["pi_slip"])
        np.testing.assert_allclose(rs["V"][0], t["V_slip"], rtol=0, atol=1e-12)


@pytest.mark.parametrize("name", table_names())
def test_vi_fp32_within_tolerance(name):
    t = load(f"table_{name}.npz")
    model = int(t["model"])
    res = oracle.value_iteration(model, cells_from_enc(t["enc"]), 0.99, 1e-6, dtype="f32")
    assert res["sweeps"] == int(t["sweeps"])  # deterministic envs converge to dv == 0 exactly
    np.testing.assert_allclose(res["V"][0], t["V"], rtol=0, atol=1e-6)
    np.testing.assert_array_equal(res["pi"][0], t["pi"])


def test_known_answer_empty16():
    # analytic KAT: V*(start) = gamma^(k-1), k = 27 actions from (1,1,dir 0) to the goal at (14,14)
    t = load("table_empty16_s0.npz")
    res = oracle.value_iteration(0, cells_from_enc(t["enc"]))
    s0 = (1 * 16 + 1) * 4 + 0
    assert res["V"][0, s0] == pytest.approx(0.99 ** 26, abs=1e-12)
    assert res["sweeps"] == 29


def test_batched_vi_global_rule():
    names = ["fourrooms_s0", "fourrooms_s1", "fourrooms_s2", "fourrooms_s3"]
    tabs = [load(f"table_{n}.npz") for n in names]
    cells = np.stack([cells_from_enc(t["enc"]) for t in tabs])
    res = oracle.value_iteration(0, cells)
    assert res["sweeps"] == max(int(t["sweeps"]) for t in tabs)
    for b, t in enumerate(tabs):
        np.testing.assert_allclose(res["V"][b], t["V"], atol=1e-12)


@pytest.mark.parametrize("slip", [None, 0.9])
@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_fixed_point_oracle_equals_literal_loop(dtype, slip):
    """orc_vi_fp (a grid at an exact fixed point is not swept again; bench.py's like-for-like CPU
    leg) against the literal global loop on every golden XYD table grid batched together: sweeps,
    V, pi and the dv trace identical; each grid's executed sweeps <= the global K."""
    names = [n for n in table_names() if int(load(f"table_{n}.npz")["model"]) == 0]
    cells = [cells_from_enc(load(f"table_{n}.npz")["enc"]) for n in names]
    shape = max(c.shape for c in cells)
    cells = [c for c in cells if c.shape == shape] or cells[:1]
    cells = np.stack(cells)
    a = oracle.value_iteration(0, cells, dtype=dtype, slip_p=slip)
    b = oracle.value_iteration(0, cells, dtype=dtype, slip_p=slip, fixed_point=True)
    assert a["sweeps"] == b["sweeps"]
    np.testing.assert_array_equal(a["V"], b["V"])
    np.testing.assert_array_equal(a["pi"], b["pi"])
    np.testing.assert_array_equal(a["dv_trace"], b["dv_trace"])
    assert b["grid_sweeps"].max() <= a["sweeps"] and b["grid_sweeps"].min() >= 1


def test_fixed_point_oracle_doorkey_golden():
    for n in table_names():
        t = load(f"table_{n}.npz")
        if int(t["model"]) != 1:
            continue
        c = cells_from_enc(t["enc"])
        b = oracle.value_iteration(1, np.stack([c, c]), dtype="f64", fixed_point=True)
        assert b["sweeps"] == int(t["sweeps"])
        np.testing.assert_array_equal(b["pi"][0], t["pi"])
        np.testing.assert_allclose(b["V"][0], t["V"], rtol=0, atol=1e-12)
        # deterministic: the grid's last swept sweep is the one that changed nothing (= K)
        assert (b["grid_sweeps"] == int(t["sweeps"])).all()


@pytest.mark.parametrize("name", traj_names())
def test_step_trajectory_matches_reference(name):
    t = load(f"traj_{name}.npz")
    for k in range(t["actions"].shape[0]):
        env = oracle.OracleEnv(t["init_enc"][k], t["init_agent"][k], int(t["max_steps"][k]),
                               SEE_THROUGH.get(name, False))
        np.testing.assert_array_equal(env.obs(), t["init_image"][k])
        for i, a in enumerate(t["actions"][k]):
            img, r, te, tr = env.step(int(a))
            ctx = f"{name} traj {k} step {i} action {a}"
            np.testing.assert_array_equal(img, t["image"][k, i], err_msg=ctx)
            assert r == t["reward"][k, i], ctx
            assert te == bool(t["terminated"][k, i]), ctx
            assert tr == bool(t["truncated"][k, i]), ctx
            assert tuple(env.state[:3]) == tuple(t["agent"][k, i]), ctx
            assert tuple(env.carry) == tuple(t["carry"][k, i]), ctx
            assert env.state[3] == t["step_count"][k, i], ctx
        np.testing.assert_array_equal(env.encode(), t["final_enc"][k])


@pytest.mark.parametrize("name", traj_names())
def test_batched_oracle_step_matches_reference(name):
    """orc_step_batch (the step path's CPU baseline) replays the reference trajectories, 4 envs at once."""
    t = load(f"traj_{name}.npz")
    n = t["actions"].shape[0]
    ob = oracle.OracleBatch(t["init_enc"], t["init_agent"], t["max_steps"], SEE_THROUGH.get(name, False))
    for i in range(t["actions"].shape[1]):
        ob.step(t["actions"][:, i])
        ctx = f"{name} step {i}"
        assert (ob.status == 0).all(), ctx
        np.testing.assert_array_equal(ob.obs, t["image"][:, i], err_msg=ctx)
        np.testing.assert_array_equal(ob.reward, t["reward"][:, i], err_msg=ctx)
        np.testing.assert_array_equal(ob.terminated, t["terminated"][:, i], err_msg=ctx)
        np.testing.assert_array_equal(ob.truncated, t["truncated"][:, i], err_msg=ctx)
        np.testing.assert_array_equal(ob.state[:, :3], t["agent"][:, i], err_msg=ctx)
        np.testing.assert_array_equal(ob.carry, t["carry"][:, i], err_msg=ctx)
    W, H = ob.W, ob.H
    for k in range(n):
        enc = np.stack([p[k, : W * H].reshape(H, W).T for p in (ob.ty, ob.co, ob.st)], axis=-1)
        np.testing.assert_array_equal(enc, t["final_enc"][k])


def test_unknown_action_raises():
    t = load("traj_empty5.npz")
    env = oracle.OracleEnv(t["init_enc"][0], t["init_agent"][0], 100, True)
    with pytest.raises(ValueError):
        env.step(7)
    assert env.state[3] == 1  # step_count is incremented before the raise (minigrid_env.py:523,579)


# ---------------------------------------------------------------------------------------------
# NoDeath lava and the finite-horizon DP, pinned by make_golden_f3.py fixtures
# ---------------------------------------------------------------------------------------------
import glob as _glob  # noqa: E402
import os as _os  # noqa: E402

from tests.golden_util import GOLDEN as _GOLDEN  # noqa: E402


def _f3(prefix):
    return sorted(_os.path.basename(p)[:-4] for p in _glob.glob(_os.path.join(_GOLDEN, prefix + "_*.npz")))


@pytest.mark.parametrize("name", _f3("nodeath"))
def test_oracle_nodeath_vs_reference_wrapper(name):
    """NoDeath(no_death_types=("lava",)) transition table through the reference wrapper and a numpy
    VI over it (wrappers.py:799-872) == the oracle's lava_mode=1 model."""
    t = load(f"{name}.npz")
    cells = cells_from_enc(t["enc"])
    dc = float(t["death_cost"])
    H, W = cells.shape
    S = W * H * 4
    # the oracle's NoDeath transition, state by state, against the reference table
    lib = oracle.lib()
    sp, dn = ctypes.c_int(0), ctypes.c_int(0)
    r = ctypes.c_double(0)
    for s in range(S):
        for a in range(7):
            ok = lib.orc_xyd_next_nodeath(oracle._ptr(cells), W, H, s, a, dc, ctypes.byref(sp), ctypes.byref(r),
                                          ctypes.byref(dn))
            if t["nxt"][s, 0] < 0:
                assert ok == 0
                continue
            assert ok == 1 and sp.value == t["nxt"][s, a] and dn.value == t["done"][s, a]
            assert r.value == t["rew"][s, a]
    o = oracle.value_iteration_ex(0, cells, dtype="f64", lava_mode=1, death_cost=dc)
    assert o["sweeps"] == int(t["sweeps"])
    np.testing.assert_array_equal(o["pi"][0], t["pi"])
    np.testing.assert_allclose(o["V"][0], t["V"], rtol=0, atol=1e-12)


@pytest.mark.parametrize("name", _f3("horizon"))
def test_oracle_finite_horizon_vs_reference_rewards(name):
    """The exact _reward() of every step_count (observed from reference step()) and a numpy
    backward induction over the reference table == the oracle's horizon mode, bit for bit."""
    t = load(f"{name}.npz")
    cells = cells_from_enc(t["enc"])
    model = int(t["model"])
    Hh = int(t["max_steps"])
    for step in range(Hh):
        assert oracle.reward(step + 1, Hh) == t["goal_reward"][step]
    for tag, g in (("g1", 1.0), ("g099", 0.99)):
        o = oracle.value_iteration_ex(model, cells, gamma=g, dtype="f64", horizon=Hh, keep_policy_t=True)
        assert o["sweeps"] == Hh
        np.testing.assert_array_equal(o["V"][0], t[f"V_{tag}"])
        np.testing.assert_array_equal(o["pi"][0], t[f"pi0_{tag}"])
        np.testing.assert_array_equal(o["pi_t"][:, 0], t[f"pi_{tag}"])


@pytest.mark.parametrize("name", table_names())
def test_numpy_restatement_matches_golden_and_oracle(name):
    """oracle/numpy_vi.py (the single-thread numpy CPU baseline) against the reference-derived
    golden V*/pi*/sweeps and bit-for-bit against the C oracle in both dtypes."""
    from oracle.numpy_vi import NumpyVI

    t = load(f"table_{name}.npz")
    model = int(t["model"])
    cells = cells_from_enc(t["enc"])
    r = NumpyVI(model, cells, dtype="f64").solve()
    assert r["sweeps"] == int(t["sweeps"])
    np.testing.assert_array_equal(r["pi"][0], t["pi"])
    np.testing.assert_allclose(r["V"][0], t["V"], rtol=0, atol=1e-12)
    for dtype in ("f32", "f64"):
        r = NumpyVI(model, cells, dtype=dtype).solve()
        o = oracle.value_iteration(model, cells, dtype=dtype)
        assert r["sweeps"] == o["sweeps"]
        np.testing.assert_array_equal(r["V"], o["V"])
        np.testing.assert_array_equal(r["pi"], o["pi"])


def _digest(a):
    import hashlib

    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest()[:8], dtype=np.uint64)[0]


def test_box_contents_trajectory_matches_reference():
    """Box(contains=...) (world_object.py:272-294) through orc_step_held: a Box's held object
    appears on toggle, travels with a carried Box and returns on drop -- every obs byte, reward,
    flag, agent, carry, carried contents and the per-step digests of encode() and of the held
    encoding equal the reference's 256-step rollouts (tests/golden/traj_box.npz, make_golden_box.py)."""
    t = load("traj_box.npz")
    for k in range(t["actions"].shape[0]):
        env = oracle.OracleEnv(t["init_enc"][k], t["init_agent"][k], int(t["max_steps"][k]), False,
                               held=t["init_held"][k])
        np.testing.assert_array_equal(env.obs(), t["init_image"][k])
        for i, a in enumerate(t["actions"][k]):
            img, r, te, tr = env.step(int(a))
            ctx = f"box traj {k} step {i} action {a}"
            np.testing.assert_array_equal(img, t["image"][k, i], err_msg=ctx)
            assert r == t["reward"][k, i] and te == bool(t["terminated"][k, i]) and tr == bool(t["truncated"][k, i]), ctx
            assert tuple(env.state[:3]) == tuple(t["agent"][k, i]), ctx
            assert tuple(env.carry) == tuple(t["carry"][k, i]), ctx
            assert tuple(env.held_carry) == tuple(t["carry_held"][k, i]), ctx
            assert _digest(env.encode()) == t["grid_digest"][k, i], ctx
            assert _digest(env.held_encoding()) == t["held_digest"][k, i], ctx
        np.testing.assert_array_equal(env.encode(), t["final_enc"][k])
        np.testing.assert_array_equal(env.held_encoding(), t["final_held"][k])


def test_box_contents_batched_oracle_matches_reference():
    t = load("traj_box.npz")
    ob = oracle.OracleBatch(t["init_enc"], t["init_agent"], t["max_steps"], False, held=t["init_held"])
    for i in range(t["actions"].shape[1]):
        ob.step(t["actions"][:, i])
        ctx = f"box step {i}"
        np.testing.assert_array_equal(ob.obs, t["image"][:, i], err_msg=ctx)
        np.testing.assert_array_equal(ob.reward, t["reward"][:, i], err_msg=ctx)
        np.testing.assert_array_equal(ob.carry, t["carry"][:, i], err_msg=ctx)
        np.testing.assert_array_equal(ob.held_carry, t["carry_held"][:, i], err_msg=ctx)
    np.testing.assert_array_equal(ob.held_encoding(), t["final_held"])


def test_without_held_planes_a_box_opens_empty():
    """The contents-free oracle (orc_step) is the reference with every Box holding nothing."""
    enc = np.zeros((5, 5, 3), np.uint8)
    enc[..., 0] = 1
    enc[0, :, 0] = enc[-1, :, 0] = enc[:, 0, 0] = enc[:, -1, 0] = 2
    enc[2, 1] = (7, 0, 0)  # a red box north of the agent
    env = oracle.OracleEnv(enc, (2, 2, 3), 100, False)
    env.step(5)
    assert env.encode()[2, 1, 0] == 1
    held = np.zeros_like(enc)
    held[2, 1] = (5, 2, 0)  # a blue key in it
    env = oracle.OracleEnv(enc, (2, 2, 3), 100, False, held=held)
    env.step(5)
    assert tuple(env.encode()[2, 1]) == (5, 2, 0) and not env.held_encoding().any()
