"""Golden trajectories for Box(contains=...) (world_object.py:272-294), from the reference itself.

Runs ONLY in the build container (reference snapshot at /root/reference, imported through the
offline gymnasium/pygame stand-in under tests/golden/shim, like make_golden.py).  No target family
places a Box that holds something, so this script builds a small room of the reference's own
classes: a walled 8x8 grid with Boxes holding a Key, a Ball, an empty Box or nothing, a locked
Door and a Goal, placed by the reference's place_obj / place_agent from np_random(seed).  Random
actions biased to pickup / drop / toggle then open, carry and drop the boxes.

    PYTHONPATH=tests/golden/shim:/root/reference PYTHONDONTWRITEBYTECODE=1 \\
        python tests/golden/make_golden_box.py

traj_box.npz: per seed the initial encode() and "held" encoding (x-major (W, H, 3): what each
Box cell holds, zeros elsewhere), agent, max_steps, actions; per step the obs image, direction,
reward (fp64), terminated, truncated, agent, carry (type, colour), carried Box contents
(type, colour, state), step_count, sha256[:8] digests of encode() and of the held encoding; the
final encode() and held encoding."""
from __future__ import annotations

import hashlib
import os

import numpy as np
from minigrid.core.grid import Grid  # noqa: E402  (reference, via the shim)
from minigrid.core.mission import MissionSpace  # noqa: E402
from minigrid.core.world_object import Ball, Box, Door, Goal, Key  # noqa: E402
from minigrid.minigrid_env import MiniGridEnv  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
SIZE = 8
COLORS = ["red", "green", "blue", "purple", "yellow", "grey"]


class BoxRoom(MiniGridEnv):
    def __init__(self, **kw):
        super().__init__(mission_space=MissionSpace(mission_func=lambda: "open the boxes"), grid_size=SIZE,
                         max_steps=4 * SIZE * SIZE, **kw)

    def _gen_grid(self, width, height):
        self.grid = Grid(width, height)
        self.grid.wall_rect(0, 0, width, height)
        for i in range(7):
            kind = self._rand_int(0, 4)
            color = COLORS[self._rand_int(0, len(COLORS))]
            inner = COLORS[self._rand_int(0, len(COLORS))]
            held = [None, Key(inner), Ball(inner), Box(inner)][kind]
            self.place_obj(Box(color, contains=held))
        self.place_obj(Door("yellow", is_locked=True))
        self.place_obj(Goal())
        self.place_agent()
        self.mission = "open the boxes"


def held_encoding(env):
    out = np.zeros((env.width, env.height, 3), np.uint8)
    for x in range(env.width):
        for y in range(env.height):
            c = env.grid.get(x, y)
            if c is not None and c.type == "box" and c.contains is not None:
                out[x, y] = c.contains.encode()
    return out


def digest(a):
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest()[:8], dtype=np.uint64)[0]


def main(n_steps=256):
    probs = np.array([0.13, 0.13, 0.24, 0.17, 0.12, 0.17, 0.04])
    keys = ("image", "direction", "reward", "terminated", "truncated", "agent", "carry", "carry_held",
            "step_count", "grid_digest", "held_digest")
    out = {k: [] for k in keys + ("seed", "max_steps", "init_image", "init_agent", "init_enc", "init_held",
                                  "actions", "final_enc", "final_held")}
    for seed in range(6):
        env = BoxRoom()
        if seed == 5:
            env.max_steps = 60
        obs, _ = env.reset(seed=seed)
        rng = np.random.default_rng(2000 + seed)
        acts = rng.choice(7, size=n_steps, p=probs).astype(np.int32)
        out["seed"].append(seed)
        out["max_steps"].append(env.max_steps)
        out["init_image"].append(obs["image"])
        out["init_agent"].append((int(env.agent_pos[0]), int(env.agent_pos[1]), int(env.agent_dir)))
        out["init_enc"].append(env.grid.encode())
        out["init_held"].append(held_encoding(env))
        rows = {k: [] for k in keys}
        for a in acts:
            obs, r, te, tr, _ = env.step(int(a))
            rows["image"].append(obs["image"])
            rows["direction"].append(int(obs["direction"]))
            rows["reward"].append(float(r))
            rows["terminated"].append(bool(te))
            rows["truncated"].append(bool(tr))
            rows["agent"].append((int(env.agent_pos[0]), int(env.agent_pos[1]), int(env.agent_dir)))
            c = env.carrying
            rows["carry"].append((0, 0) if c is None else tuple(int(v) for v in c.encode()[:2]))
            ch = (0, 0, 0)
            if c is not None and c.type == "box" and c.contains is not None:
                ch = tuple(int(v) for v in c.contains.encode())
            rows["carry_held"].append(ch)
            rows["step_count"].append(env.step_count)
            rows["grid_digest"].append(digest(env.grid.encode()))
            rows["held_digest"].append(digest(held_encoding(env)))
        out["actions"].append(acts)
        out["final_enc"].append(env.grid.encode())
        out["final_held"].append(held_encoding(env))
        for k, v in rows.items():
            out[k].append(v)
    dt = {"reward": np.float64, "grid_digest": np.uint64, "held_digest": np.uint64, "image": np.uint8,
          "init_image": np.uint8, "init_enc": np.uint8, "init_held": np.uint8, "final_enc": np.uint8,
          "final_held": np.uint8, "terminated": np.uint8, "truncated": np.uint8}
    arrs = {k: np.array(v, dt.get(k, np.int32)) for k, v in out.items()}
    np.savez_compressed(os.path.join(HERE, "traj_box.npz"), **arrs)
    opened = int(((arrs["init_enc"][..., 0] == 7).sum() - (arrs["final_enc"][..., 0] == 7).sum()))
    print("traj box", {k: v.shape for k, v in arrs.items()}, "boxes gone by the end:", opened, flush=True)


if __name__ == "__main__":
    main()
