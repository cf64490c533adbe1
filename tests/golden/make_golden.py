"""Generate the golden vectors that pin the oracle and the HIP path to the reference.

Runs ONLY in the build container, where the read-only reference snapshot lives at
/root/reference.  The reference is imported through the offline gymnasium/pygame stand-in under
tests/golden/shim (gymnasium and pygame are not installed).  Nothing
from the reference is copied: this script calls the reference's own classes and stores what they
return as small .npz fixtures next to this file.  The GPU box never runs this script.

    PYTHONPATH=tests/golden/shim:/root/reference PYTHONDONTWRITEBYTECODE=1 \
        python tests/golden/make_golden.py

What is captured (every value comes out of the reference's own code):
  grids_<env>.npz      reset(seed) for seeds 0..63: grid.encode() (W,H,3) x-major + agent x,y,dir
  digests.json         sha256 over encode().tobytes() || int32[x,y,dir] for large seed ranges
  traj_<env>.npz       256-step trajectories of env.step() with seeded random actions:
                       obs image, dir, reward (fp64), terminated, truncated, agent, carrying,
                       per-step grid digest
  table_<env>_s<seed>.npz
                       the MDP transition table extracted by driving reference step() from every
                       enumerated state (conventions: DESIGN.md "A9"), plus V*, pi*, sweeps of a
                       numpy Jacobi value iteration over that table (deterministic and slip p=0.9).
"""
from __future__ import annotations

import copy
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

from minigrid.core.world_object import Key  # noqa: E402  (reference, via the shim)
from minigrid.envs import CrossingEnv, DoorKeyEnv, EmptyEnv, FourRoomsEnv  # noqa: E402

ENVS = {
    "empty5": lambda: EmptyEnv(size=5),
    "empty16": lambda: EmptyEnv(size=16),
    "fourrooms": lambda: FourRoomsEnv(),
    "lava9n1": lambda: CrossingEnv(size=9, num_crossings=1),
    "lava11n5": lambda: CrossingEnv(size=11, num_crossings=5),
    "doorkey5": lambda: DoorKeyEnv(size=5),
    "doorkey8": lambda: DoorKeyEnv(size=8),
    "doorkey16": lambda: DoorKeyEnv(size=16),
}

GAMMA = 0.99
TOL = 1e-6
SLIP_P = 0.9
DK_ACTIONS = (0, 1, 2, 3, 5)  # DoorKey DP action lanes -> env actions (left,right,fwd,pickup,toggle)


def agent_xyd(env):
    return int(env.agent_pos[0]), int(env.agent_pos[1]), int(env.agent_dir)


def grid_digest_bytes(env):
    x, y, d = agent_xyd(env)
    return env.grid.encode().tobytes() + np.array([x, y, d], dtype=np.int32).tobytes()


# ----------------------------------------------------------------------------------------------
# 1. grids + digests
# ----------------------------------------------------------------------------------------------
def gen_grids():
    for name in ("empty5", "empty16", "fourrooms", "lava11n5", "doorkey16", "doorkey8"):
        env = ENVS[name]()
        encs, agents = [], []
        for seed in range(64):
            env.reset(seed=seed)
            encs.append(env.grid.encode())
            agents.append(agent_xyd(env))
        np.savez_compressed(os.path.join(HERE, f"grids_{name}.npz"),
                            enc=np.stack(encs), agent=np.array(agents, dtype=np.int32))


def gen_digests():
    # the BASELINE batch sizes: FourRooms x 4096 (configs[2]), LavaS11N5 x 65536 (configs[3]),
    # DoorKey-16 x 65536 (configs[4], SURVEY 8(d) cfg 5)
    digests = {}
    for name, n in (("fourrooms", 4096), ("lava11n5", 65536), ("doorkey16", 65536)):
        env = ENVS[name]()
        h = hashlib.sha256()
        for seed in range(n):
            env.reset(seed=seed)
            h.update(grid_digest_bytes(env))
        digests[name] = {"seeds": n, "sha256": h.hexdigest()}
        print("digest", name, n, h.hexdigest()[:16], flush=True)
    with open(os.path.join(HERE, "digests.json"), "w") as f:
        json.dump(digests, f, indent=1)


# ----------------------------------------------------------------------------------------------
# 2. step trajectories
# ----------------------------------------------------------------------------------------------
def carry_code(env):
    c = env.carrying
    if c is None:
        return (0, 0)
    t, col, _ = c.encode()
    return (int(t), int(col))


def policy_state(env, name):
    """State index of the env's current configuration under the A9 conventions (None if the
    configuration is outside the model, e.g. a dropped key)."""
    x, y, d = agent_xyd(env)
    W = env.width
    s = (y * W + x) * 4 + d
    if not name.startswith("doorkey"):
        return s
    enc = env.grid.encode()
    door = np.argwhere(enc[:, :, 0] == 4)[0]
    dstate = enc[door[0], door[1], 2]
    hk = 1 if env.carrying is not None else 0
    if not hk and not (enc[:, :, 0] == 5).any():
        return None
    if hk and (enc[:, :, 0] == 5).any():
        return None
    do = 1 if dstate == 0 else 0
    return (s * 2 + hk) * 2 + do


def gen_trajectories(n_steps=256):
    for name in ENVS:
        out = {k: [] for k in ("seed", "init_image", "init_agent", "init_enc", "actions", "image",
                               "direction", "reward", "terminated", "truncated", "agent",
                               "carry", "step_count", "grid_digest", "final_enc", "max_steps")}
        for seed in range(4):
            env = ENVS[name]()
            if seed == 3:
                env.max_steps = 40  # exercise truncation (tests/test_envs.py:146-166 idea)
            obs, _ = env.reset(seed=seed)
            rng = np.random.default_rng(1000 + seed)
            acts = rng.integers(0, 7, size=n_steps)
            pol = None
            if seed == 2:  # epsilon-greedy on the table policy: reaches goals, opens doors
                probe = ENVS[name]()
                probe.reset(seed=seed)
                if name.startswith("doorkey"):
                    _, nxt, rew, done = doorkey_table(probe)
                else:
                    _, nxt, rew, done = xyd_table(probe)
                pol = numpy_vi(nxt, rew, done, GAMMA, TOL)[1]
                explore = rng.random(n_steps) < 0.2
            out["seed"].append(seed)
            out["max_steps"].append(env.max_steps)
            out["init_image"].append(obs["image"])
            out["init_agent"].append(agent_xyd(env))
            out["init_enc"].append(env.grid.encode())
            rows = {k: [] for k in ("image", "direction", "reward", "terminated", "truncated",
                                    "agent", "carry", "step_count", "grid_digest")}
            acts = acts.copy()
            for i in range(n_steps):
                if pol is not None and not explore[i]:
                    si = policy_state(env, name)
                    if si is not None and pol[si] >= 0:
                        acts[i] = DK_ACTIONS[pol[si]] if name.startswith("doorkey") else pol[si]
                a = acts[i]
                obs, r, te, tr, _ = env.step(int(a))
                rows["image"].append(obs["image"])
                rows["direction"].append(int(obs["direction"]))
                rows["reward"].append(float(r))
                rows["terminated"].append(bool(te))
                rows["truncated"].append(bool(tr))
                rows["agent"].append(agent_xyd(env))
                rows["carry"].append(carry_code(env))
                rows["step_count"].append(env.step_count)
                dg = hashlib.sha256(env.grid.encode().tobytes()).digest()[:8]
                rows["grid_digest"].append(np.frombuffer(dg, dtype=np.uint64)[0])
            out["actions"].append(acts.astype(np.int32))
            out["final_enc"].append(env.grid.encode())
            for k, v in rows.items():
                out[k].append(v)
        arrs = {
            "seed": np.array(out["seed"], np.int32),
            "max_steps": np.array(out["max_steps"], np.int32),
            "init_image": np.stack(out["init_image"]).astype(np.uint8),
            "init_agent": np.array(out["init_agent"], np.int32),
            "init_enc": np.stack(out["init_enc"]).astype(np.uint8),
            "final_enc": np.stack(out["final_enc"]).astype(np.uint8),
            "actions": np.stack(out["actions"]),
            "image": np.array(out["image"], np.uint8),
            "direction": np.array(out["direction"], np.int32),
            "reward": np.array(out["reward"], np.float64),
            "terminated": np.array(out["terminated"], np.uint8),
            "truncated": np.array(out["truncated"], np.uint8),
            "agent": np.array(out["agent"], np.int32),
            "carry": np.array(out["carry"], np.int32),
            "step_count": np.array(out["step_count"], np.int32),
            "grid_digest": np.array(out["grid_digest"], np.uint64),
        }
        np.savez_compressed(os.path.join(HERE, f"traj_{name}.npz"), **arrs)
        print("traj", name, flush=True)


# ----------------------------------------------------------------------------------------------
# 3. transition tables through reference step(), and a numpy Jacobi VI over them
# ----------------------------------------------------------------------------------------------
FREE = (1, 3)  # empty, floor


def xyd_table(env):
    W, H = env.width, env.height
    enc = env.grid.encode()
    S = W * H * 4
    nxt = np.full((S, 7), -1, np.int32)
    rew = np.zeros((S, 7), np.float64)
    done = np.zeros((S, 7), np.uint8)
    for y in range(H):
        for x in range(W):
            if enc[x, y, 0] not in FREE:
                continue
            for d in range(4):
                s = (y * W + x) * 4 + d
                for a in range(7):
                    env.agent_pos = (x, y)
                    env.agent_dir = d
                    env.step_count = 0
                    env.carrying = None
                    _, r, te, _, _ = env.step(a)
                    nx, ny, nd = agent_xyd(env)
                    nxt[s, a] = (ny * W + nx) * 4 + nd
                    cell = env.grid.get(nx, ny)
                    done[s, a] = 1 if te else 0
                    rew[s, a] = 1.0 if (te and cell is not None and cell.type == "goal") else 0.0
                    assert (r > 0) == (rew[s, a] > 0)
    return enc, nxt, rew, done


def doorkey_table(env):
    W, H = env.width, env.height
    enc0 = env.grid.encode()
    kpos = tuple(int(v) for v in np.argwhere(enc0[:, :, 0] == 5)[0])
    dpos = tuple(int(v) for v in np.argwhere(enc0[:, :, 0] == 4)[0])
    key = env.grid.get(*kpos)
    door = env.grid.get(*dpos)
    assert isinstance(key, Key) and door.is_locked and key.color == door.color
    S = W * H * 16
    nxt = np.full((S, 5), -1, np.int32)
    rew = np.zeros((S, 5), np.float64)
    done = np.zeros((S, 5), np.uint8)
    for y in range(H):
        for x in range(W):
            t = enc0[x, y, 0]
            for hk in (0, 1):
                for do in (0, 1):
                    ok = (t in FREE) or (t == 4 and do == 1) or (t == 5 and hk == 1)
                    if not ok:
                        continue
                    for d in range(4):
                        s = (((y * W + x) * 4 + d) * 2 + hk) * 2 + do
                        for li, a in enumerate(DK_ACTIONS):
                            env.grid.set(*kpos, None if hk else key)
                            env.carrying = key if hk else None
                            door.is_open = bool(do)
                            door.is_locked = not do
                            env.agent_pos = (x, y)
                            env.agent_dir = d
                            env.step_count = 0
                            _, r, te, _, _ = env.step(a)
                            nx, ny, nd = agent_xyd(env)
                            nhk = 1 if env.carrying is not None else 0
                            if not nhk:
                                assert env.grid.get(*kpos) is key
                            ndo = 1 if door.is_open else 0
                            nxt[s, li] = (((ny * W + nx) * 4 + nd) * 2 + nhk) * 2 + ndo
                            cell = env.grid.get(nx, ny)
                            done[s, li] = 1 if te else 0
                            rew[s, li] = 1.0 if (te and cell is not None and cell.type == "goal") else 0.0
    # restore reset configuration
    env.grid.set(*kpos, key)
    env.carrying = None
    door.is_open, door.is_locked = False, True
    return enc0, nxt, rew, done


def numpy_vi(nxt, rew, done, gamma, tol, slip_p=None, max_sweeps=10000):
    """Jacobi value iteration with the build's A9 conventions, written independently of oracle/.

    Q_det[s,a] = R + gamma*(1-done)*V[s'];  slip: Q[s,a] = p*Q_det[s,a] + c*(((((Q0+Q1)+Q2)+Q3)+Q4)+Q5)
    with c = (1-p)/6.  V_{k+1} = max_a Q (lowest index wins ties).  Stop after sweep k when
    max|V_k - V_{k-1}| < tol.  Invalid (absorbing) states keep V=0 and pi=-1.
    """
    S, A = nxt.shape
    valid = nxt[:, 0] >= 0
    V = np.zeros(S, np.float64)
    safe = np.where(nxt >= 0, nxt, 0)
    g = np.float64(gamma)
    k = 0
    while True:
        k += 1
        Vn = V[safe]
        qd = np.where(done.astype(bool), rew, rew + g * Vn)
        if slip_p is not None:
            p = np.float64(slip_p)
            c = (1.0 - p) / 6.0
            s6 = qd[:, 0] + qd[:, 1]
            for j in range(2, 6):
                s6 = s6 + qd[:, j]
            q = p * qd + (c * s6)[:, None]
        else:
            q = qd
        newV = np.where(valid, q.max(axis=1), 0.0)
        pi = np.where(valid, q.argmax(axis=1), -1).astype(np.int8)
        dv = float(np.max(np.abs(newV - V)))
        V = newV
        if dv < tol or k >= max_sweeps:
            return V, pi, k, dv


def gen_tables():
    jobs = [("empty5", [0]), ("empty16", [0]), ("fourrooms", [0, 1, 2, 3]),
            ("lava11n5", [0, 1, 2, 3]), ("lava9n1", [2]), ("doorkey16", [0, 1]), ("doorkey8", [0, 1, 2])]
    summary = {}
    for name, seeds in jobs:
        for seed in seeds:
            env = ENVS[name]()
            env.reset(seed=seed)
            start = agent_xyd(env)
            if name.startswith("doorkey"):
                enc, nxt, rew, done = doorkey_table(env)
                model = 1
            else:
                enc, nxt, rew, done = xyd_table(env)
                model = 0
            V, pi, k, dv = numpy_vi(nxt, rew, done, GAMMA, TOL)
            out = dict(enc=enc, start=np.array(start, np.int32), nxt=nxt, rew=rew, done=done,
                       model=np.int32(model), V=V, pi=pi, sweeps=np.int32(k), dv=np.float64(dv))
            W = enc.shape[0]
            s0 = (start[1] * W + start[0]) * 4 + start[2]
            if model == 1:
                s0 = s0 * 4
            entry = {"sweeps": k, "V_start": float(V[s0])}
            if model == 0:
                Vs, pis, ks, dvs = numpy_vi(nxt, rew, done, GAMMA, TOL, slip_p=SLIP_P)
                out.update(V_slip=Vs, pi_slip=pis, sweeps_slip=np.int32(ks), dv_slip=np.float64(dvs))
                entry["sweeps_slip"] = ks
                entry["V_slip_start"] = float(Vs[s0])
            np.savez_compressed(os.path.join(HERE, f"table_{name}_s{seed}.npz"), **out)
            summary[f"{name}_s{seed}"] = entry
            print("table", name, seed, entry, flush=True)
    with open(os.path.join(HERE, "tables_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)


if __name__ == "__main__":
    what = sys.argv[1:] or ["grids", "traj", "tables"]  # or "digests" alone
    if "tables" in what:
        gen_tables()
    if "traj" in what:
        gen_trajectories()
    if "grids" in what:
        gen_grids()
    if "grids" in what or "digests" in what:
        gen_digests()
