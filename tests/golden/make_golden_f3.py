"""Golden vectors for the SURVEY 8(f) item-3 DP options, captured from the reference itself.

Runs ONLY in the build container (the reference is imported through the offline shim, exactly
like make_golden.py, whose table/VI helpers this script reuses):

    PYTHONPATH=tests/golden/shim:/root/reference:tests/golden PYTHONDONTWRITEBYTECODE=1 \
        python tests/golden/make_golden_f3.py

What is captured:
  grids_<env>.npz / digests_f3.json   reset(seed) of the sibling envs with the same cell types:
                       LavaGapS5/6/7 (lavagap.py:101-136) and DistShift1/2 (distshift.py:99-121)
  table_<env>_s<seed>.npz             their transition tables through reference step() + numpy VI
  nodeath_<env>_s<seed>.npz           the table through NoDeath(env, ("lava",), death_cost)
                       (wrappers.py:799-872): lava cells become states, entering lava gives
                       death_cost without termination; numpy VI over it
  horizon_<env>_s<seed>.npz           finite-horizon DP over step_count: the reward of entering the
                       goal observed from reference step() at every step_count t = 0..H-1 (the
                       exact _reward(), minigrid_env.py:235-240), truncation observed at t = H-1,
                       and a numpy backward induction (gamma = 1 and 0.99) over it
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

import make_golden as mg0  # noqa: E402  (tests/golden on PYTHONPATH)
from minigrid.envs import CrossingEnv, DistShiftEnv, DoorKeyEnv, EmptyEnv, FourRoomsEnv, LavaGapEnv  # noqa: E402
from minigrid.wrappers import NoDeath  # noqa: E402

HERE = mg0.HERE
SIB = {
    "lavagap5": lambda: LavaGapEnv(size=5),
    "lavagap6": lambda: LavaGapEnv(size=6),
    "lavagap7": lambda: LavaGapEnv(size=7),
    "distshift1": lambda: DistShiftEnv(strip2_row=2),
    "distshift2": lambda: DistShiftEnv(strip2_row=5),
}
DEATH_COST = -1.0


def gen_sibling():
    digests = {}
    for name, ctor in SIB.items():
        env = ctor()
        encs, agents = [], []
        for seed in range(64):
            env.reset(seed=seed)
            encs.append(env.grid.encode())
            agents.append(mg0.agent_xyd(env))
        np.savez_compressed(os.path.join(HERE, f"grids_{name}.npz"), enc=np.stack(encs),
                            agent=np.array(agents, np.int32), max_steps=np.int32(env.max_steps),
                            see_through=np.uint8(env.see_through_walls))
    env = SIB["lavagap7"]()
    h = hashlib.sha256()
    for seed in range(4096):
        env.reset(seed=seed)
        h.update(mg0.grid_digest_bytes(env))
    digests["lavagap7"] = {"seeds": 4096, "sha256": h.hexdigest()}
    with open(os.path.join(HERE, "digests_f3.json"), "w") as f:
        json.dump(digests, f, indent=1)
    for name, seed in (("lavagap5", 0), ("lavagap7", 3), ("distshift1", 0), ("distshift2", 0)):
        env = SIB[name]()
        env.reset(seed=seed)
        enc, nxt, rew, done = mg0.xyd_table(env)
        V, pi, k, dv = mg0.numpy_vi(nxt, rew, done, mg0.GAMMA, mg0.TOL)
        Vs, pis, ks, dvs = mg0.numpy_vi(nxt, rew, done, mg0.GAMMA, mg0.TOL, slip_p=mg0.SLIP_P)
        np.savez_compressed(os.path.join(HERE, f"table_{name}_s{seed}.npz"), enc=enc,
                            start=np.array(mg0.agent_xyd(env), np.int32), nxt=nxt, rew=rew, done=done,
                            model=np.int32(0), V=V, pi=pi, sweeps=np.int32(k), dv=np.float64(dv),
                            V_slip=Vs, pi_slip=pis, sweeps_slip=np.int32(ks), dv_slip=np.float64(dvs))
        print("sibling table", name, seed, k, flush=True)


def nodeath_table(env, death_cost):
    """Drive NoDeath(env).step from every (x, y, dir) whose cell the agent may occupy under the
    wrapper (empty / floor / lava)."""
    wrapped = NoDeath(env, no_death_types=("lava",), death_cost=death_cost)
    W, H = env.width, env.height
    enc = env.grid.encode()
    S = W * H * 4
    nxt = np.full((S, 7), -1, np.int32)
    rew = np.zeros((S, 7), np.float64)
    done = np.zeros((S, 7), np.uint8)
    for y in range(H):
        for x in range(W):
            if enc[x, y, 0] not in (1, 3, 9):
                continue
            for d in range(4):
                s = (y * W + x) * 4 + d
                for a in range(7):
                    env.agent_pos = (x, y)
                    env.agent_dir = d
                    env.step_count = 0
                    env.carrying = None
                    _, r, te, _, _ = wrapped.step(a)
                    nx, ny, nd = mg0.agent_xyd(env)
                    nxt[s, a] = (ny * W + nx) * 4 + nd
                    cell = env.grid.get(nx, ny)
                    goal = te and cell is not None and cell.type == "goal"
                    done[s, a] = 1 if te else 0
                    rew[s, a] = 1.0 if goal else float(r)  # 0, or 0 + death_cost from the wrapper
    return enc, nxt, rew, done


def gen_nodeath():
    # the wrapper's own doctest env: LavaCrossingS9N1 seed 2, right then forward into lava
    env = CrossingEnv(size=9, num_crossings=1)
    w = NoDeath(env, no_death_types=("lava",), death_cost=DEATH_COST)
    w.reset(seed=2)
    w.step(1)
    _, r, te, *_ = w.step(2)
    assert (r, te) == (DEATH_COST, False), (r, te)
    for name, ctor, seed in (("lava9n1", lambda: CrossingEnv(size=9, num_crossings=1), 2),
                             ("lava11n5", lambda: CrossingEnv(size=11, num_crossings=5), 0),
                             ("lavagap7", SIB["lavagap7"], 3),
                             ("distshift1", SIB["distshift1"], 0)):
        env = ctor()
        env.reset(seed=seed)
        enc, nxt, rew, done = nodeath_table(env, DEATH_COST)
        V, pi, k, dv = mg0.numpy_vi(nxt, rew, done, mg0.GAMMA, mg0.TOL)
        np.savez_compressed(os.path.join(HERE, f"nodeath_{name}_s{seed}.npz"), enc=enc,
                            start=np.array(mg0.agent_xyd(env), np.int32), nxt=nxt, rew=rew, done=done,
                            death_cost=np.float64(DEATH_COST), V=V, pi=pi, sweeps=np.int32(k),
                            dv=np.float64(dv))
        print("nodeath table", name, seed, k, float(V.min()), float(V.max()), flush=True)


def goal_rewards(env, table):
    """Reward and truncation reference step() returns when entering the goal from step_count t,
    for every t in [0, max_steps): the exact _reward() at step_count t + 1."""
    nxt, rew, done = table
    s, a = map(int, np.argwhere((done == 1) & (rew == 1.0))[0])
    W = env.width
    A = nxt.shape[1]
    c, rest = divmod(s, 4 if A == 7 else 16)
    x, y = c % W, c // W
    d = rest if A == 7 else rest >> 2
    act = a if A == 7 else mg0.DK_ACTIONS[a]
    out = np.zeros(env.max_steps, np.float64)
    trunc = np.zeros(env.max_steps, np.uint8)
    for t in range(env.max_steps):
        env.agent_pos, env.agent_dir, env.step_count = (x, y), d, t
        _, r, te, tr, _ = env.step(act)
        assert te
        out[t] = r
        trunc[t] = tr
    return out, trunc


def numpy_horizon(nxt, rew, done, rgoal, gamma):
    """Backward induction V_H = 0, V_t = max_a (done ? R_t : R_t + gamma * V_{t+1}[s'])."""
    S, A = nxt.shape
    valid = nxt[:, 0] >= 0
    safe = np.where(nxt >= 0, nxt, 0)
    Hh = len(rgoal)
    V = np.zeros(S, np.float64)
    pis = np.zeros((Hh, S), np.int8)
    goal = (done == 1) & (rew == 1.0)
    for t in range(Hh - 1, -1, -1):
        R = np.where(goal, rgoal[t], rew)
        q = np.where(done.astype(bool), R, R + gamma * V[safe])
        Vn = np.where(valid, q.max(axis=1), 0.0)
        pis[t] = np.where(valid, q.argmax(axis=1), -1)
        V = Vn
    return V, pis


def gen_horizon():
    jobs = (("empty5", lambda: EmptyEnv(size=5), 0, "xyd"),
            ("lava9n1", lambda: CrossingEnv(size=9, num_crossings=1), 2, "xyd"),
            ("fourrooms", lambda: FourRoomsEnv(), 0, "xyd"),
            ("lavagap5", SIB["lavagap5"], 1, "xyd"),
            ("doorkey5", lambda: DoorKeyEnv(size=5), 0, "doorkey"))
    for name, ctor, seed, model in jobs:
        env = ctor()
        env.reset(seed=seed)
        start = mg0.agent_xyd(env)
        if model == "doorkey":
            enc, nxt, rew, done = mg0.doorkey_table(env)
        else:
            enc, nxt, rew, done = mg0.xyd_table(env)
        rg, tr = goal_rewards(env, (nxt, rew, done))
        assert tr[-1] == 1 and not tr[:-1].any()
        out = dict(enc=enc, start=np.array(start, np.int32), nxt=nxt, rew=rew, done=done,
                   model=np.int32(0 if model == "xyd" else 1), max_steps=np.int32(env.max_steps),
                   goal_reward=rg, truncated=tr)
        for tag, g in (("g1", 1.0), ("g099", mg0.GAMMA)):
            V, pis = numpy_horizon(nxt, rew, done, rg, g)
            out[f"V_{tag}"] = V
            out[f"pi0_{tag}"] = pis[0]
            out[f"pi_{tag}"] = pis  # (H, S) int8
        np.savez_compressed(os.path.join(HERE, f"horizon_{name}_s{seed}.npz"), **out)
        print("horizon", name, seed, env.max_steps, flush=True)


if __name__ == "__main__":
    gen_sibling()
    gen_nodeath()
    gen_horizon()
