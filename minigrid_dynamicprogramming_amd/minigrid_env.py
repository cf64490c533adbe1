"""MiniGridEnv: the gymnasium Env surface of the reference, stepped by the HIP engine.

Drop-in for minigrid/minigrid_env.py:24-784 (MiniGridEnv) on the hot path:
  reset(*, seed, options) -> (obs, {})                     minigrid_env.py:119-157
  step(action) -> (obs, reward, terminated, truncated, {})  minigrid_env.py:520-590
  obs = {"image": uint8 (V,V,3), "direction": int, "mission": str}  (:629-645)
Grid generation (`_gen_grid`, the RNG helpers and placement, :242-390) runs on the host with the
same numpy PCG64 stream as gymnasium seeding, so grids are identical to the reference's
(pinned by tests/test_host_envs.py against reference digests).  Every step and observation runs
in libmgdp.so on the GPU (csrc/envs.hip); there is no CPU stepping path.

Attributes callers and wrappers read (agent_pos, agent_dir, carrying, grid, step_count, ...) are
mirrored lazily from HBM; assigning them, or editing env.grid, pushes the change back before the
next step.
"""
from __future__ import annotations

import ctypes
import math
from abc import abstractmethod
from typing import Any, Iterable, TypeVar

import numpy as np

from . import _lib
from ._gym import Env, spaces
from .core import COLOR_NAMES, DIR_TO_VEC, OBJECT_TO_IDX, Actions, Grid, WorldObj

T = TypeVar("T")


class MissionSpace(spaces.Space):
    """Constant-mission space (the target envs use constant strings; minigrid/core/mission.py)."""

    def __init__(self, mission_func, ordered_placeholders=None, seed=None):
        self.mission_func = mission_func
        self.ordered_placeholders = ordered_placeholders
        super().__init__(dtype=str, seed=seed)

    def sample(self) -> str:
        if self.ordered_placeholders is None:
            return self.mission_func()
        ph = [lst[self.np_random.integers(0, len(lst))] for lst in self.ordered_placeholders]
        return self.mission_func(*ph)

    def contains(self, x) -> bool:
        return isinstance(x, str)


class _DeviceEnv:
    """One env resident on one GPU (an mgdp_envs handle with B = 1)."""

    def __init__(self, W: int, H: int, view: int, device: int = 0):
        self.L = _lib.load()
        _lib.require_gpu()
        h = ctypes.c_void_p()
        _lib.check(self.L.mgdp_envs_create(device, 1, W, H, view, ctypes.byref(h)), "mgdp_envs_create")
        self.h = h
        self.W, self.H, self.view = W, H, view
        self.obs = np.zeros((1, view, view, 3), np.uint8)
        self.dir = np.zeros(1, np.int32)
        self.rew = np.zeros(1, np.float64)
        self.term = np.zeros(1, np.uint8)
        self.trunc = np.zeros(1, np.uint8)
        self.status = np.zeros(1, np.int32)
        self.act = np.zeros(1, np.int32)
        self.held = False  # Box contents planes in use on the device

    def __del__(self):
        try:
            if getattr(self, "h", None):
                self.L.mgdp_envs_destroy(self.h)
                self.h = None
        except Exception:
            pass


class MiniGridEnv(Env):
    metadata = {"render_modes": ["human", "rgb_array"], "render_fps": 10}

    def __init__(
        self,
        mission_space: MissionSpace,
        grid_size: int | None = None,
        width: int | None = None,
        height: int | None = None,
        max_steps: int = 100,
        see_through_walls: bool = False,
        agent_view_size: int = 7,
        render_mode: str | None = None,
        screen_size: int | None = 640,
        highlight: bool = True,
        tile_size: int = 32,
        agent_pov: bool = False,
        device: int = 0,
    ):
        self.mission = mission_space.sample()
        if grid_size:
            assert width is None and height is None
            width = grid_size
            height = grid_size
        assert width is not None and height is not None
        self.actions = Actions
        self.action_space = spaces.Discrete(len(self.actions))
        assert agent_view_size % 2 == 1
        assert agent_view_size >= 3
        self.agent_view_size = agent_view_size
        image_space = spaces.Box(low=0, high=255, shape=(agent_view_size, agent_view_size, 3), dtype="uint8")
        self.observation_space = spaces.Dict(
            {"image": image_space, "direction": spaces.Discrete(4), "mission": mission_space})
        self.reward_range = (0, 1)
        self.screen_size = screen_size
        self.render_mode = render_mode
        self.highlight = highlight
        self.tile_size = tile_size
        self.agent_pov = agent_pov
        self.width = width
        self.height = height
        assert isinstance(max_steps, int), f"The argument max_steps must be an integer, got: {type(max_steps)}"
        self.max_steps = max_steps
        self.see_through_walls = see_through_walls
        self.device = device
        # host mirror of the env state (authoritative copy lives in HBM after reset)
        self._agent_pos = None
        self._agent_dir = None
        self._carrying = None
        self._step_count = 0
        self._grid = Grid(width, height)
        self._dev: _DeviceEnv | None = None
        self._host_stale = False   # HBM changed since the last pull
        self._push_pending = False  # host edits not yet in HBM
        self._generating = False

    # ------------------------------------------------------------------ state mirroring
    def _pull(self):
        if not self._host_stale or self._dev is None:
            return
        enc = np.zeros((1, self.width, self.height, 3), np.uint8)
        agent = np.zeros((1, 3), np.int32)
        carry = np.zeros((1, 2), np.int32)
        sc = np.zeros(1, np.int32)
        d = self._dev
        _lib.check(d.L.mgdp_envs_get_state(d.h, _lib.ptr(enc), _lib.ptr(agent), _lib.ptr(carry), _lib.ptr(sc)),
                   "mgdp_envs_get_state")
        self._host_stale = False
        owner, self._grid._owner = self._grid._owner, None
        self._grid.load_encoding(enc[0])
        held = np.zeros((1, self.width, self.height, 3), np.uint8)
        carry_held = np.zeros((1, 3), np.int32)
        if d.held:
            _lib.check(d.L.mgdp_envs_get_contents(d.h, _lib.ptr(held), _lib.ptr(carry_held)), "mgdp_envs_get_contents")
            self._grid.load_held(held[0])
        self._grid._owner = owner
        self._agent_pos = (int(agent[0, 0]), int(agent[0, 1]))
        self._agent_dir = int(agent[0, 2])
        self._step_count = int(sc[0])
        if carry[0, 0] > 0:
            c = self._carrying
            if c is None or c.encode()[:2] != (int(carry[0, 0]), int(carry[0, 1])):
                c = WorldObj.decode(int(carry[0, 0]), int(carry[0, 1]), 0)
                c.cur_pos = np.array([-1, -1])
            if d.held and c.type == "box":  # what the carried Box holds
                c.contains = WorldObj.decode(*carry_held[0]) if carry_held[0, 0] > OBJECT_TO_IDX["empty"] else None
            self._carrying = c
        else:
            self._carrying = None

    def _grid_edited(self):
        if not self._generating:
            self._push_pending = True

    def _ensure_device(self):
        if self._dev is None:
            self._dev = _DeviceEnv(self.width, self.height, self.agent_view_size, self.device)

    def _push(self):
        """Upload the host grid + agent state to HBM."""
        self._ensure_device()
        d = self._dev
        enc = np.ascontiguousarray(self._grid.encode()[None])
        ap = self._agent_pos
        agent = np.array([[int(ap[0]), int(ap[1]), int(self._agent_dir)]], np.int32)
        ms = np.array([self.max_steps], np.int32)
        see = np.array([1 if self.see_through_walls else 0], np.uint8)
        _lib.check(d.L.mgdp_envs_load(d.h, _lib.ptr(enc), _lib.ptr(agent), _lib.ptr(ms), _lib.ptr(see), None),
                   "mgdp_envs_load")
        carry = np.zeros((1, 2), np.int32)
        if self._carrying is not None:
            t, c, _ = self._carrying.encode()
            carry[0] = (t, c)
        sc = np.array([self._step_count], np.int32)
        _lib.check(d.L.mgdp_envs_set_state(d.h, None, _lib.ptr(carry), _lib.ptr(sc), None), "mgdp_envs_set_state")
        held = self._grid.encode_held()
        carry_held = np.zeros((1, 3), np.int32)
        inner = getattr(self._carrying, "contains", None) if self._carrying is not None else None
        if inner is not None:
            if self._carrying.type != "box" or getattr(inner, "contains", None) is not None:
                raise NotImplementedError("only a Box holds an object, and a held Box holds nothing")
            carry_held[0] = inner.encode()
        if d.held or held.any() or carry_held.any():  # Box(contains=...) in play: the contents planes
            _lib.check(d.L.mgdp_envs_set_contents(d.h, _lib.ptr(np.ascontiguousarray(held[None])), _lib.ptr(carry_held)),
                       "mgdp_envs_set_contents")
            d.held = True
        self._push_pending = False

    def _sync_to_device(self):
        if self._push_pending or self._dev is None:
            self._push()

    def _attr_set(self, name, value):
        self._pull()
        setattr(self, name, value)
        self._push_pending = True

    agent_pos = property(lambda self: (self._pull(), self._agent_pos)[1],
                         lambda self, v: self._attr_set("_agent_pos", v))
    agent_dir = property(lambda self: (self._pull(), self._agent_dir)[1],
                         lambda self, v: self._attr_set("_agent_dir", v))
    carrying = property(lambda self: (self._pull(), self._carrying)[1],
                        lambda self, v: self._attr_set("_carrying", v))
    step_count = property(lambda self: (self._pull(), self._step_count)[1],
                          lambda self, v: self._attr_set("_step_count", v))

    @property
    def grid(self) -> Grid:
        self._pull()
        return self._grid

    @grid.setter
    def grid(self, g: Grid):
        self._pull()
        g._owner = self
        self._grid = g
        if not self._generating:
            self._push_pending = True

    # ------------------------------------------------------------------ reset / step
    def reset(self, *, seed: int | None = None, options: dict[str, Any] | None = None):
        self.generate(seed=seed)
        self._push()
        return self.gen_obs(), {}

    def generate(self, seed: int | None = None):
        """Host half of reset(): seed the RNG and run _gen_grid (no device work).

        Returns (enc, agent): the reference's Grid.encode() (W, H, 3) and (x, y, dir).  Used to build
        large DP batches from seeds without a device env per grid."""
        super().reset(seed=seed)
        self._host_stale = False
        self._agent_pos = (-1, -1)
        self._agent_dir = -1
        self._generating = True
        try:
            self._gen_grid(self.width, self.height)
        finally:
            self._generating = False
        self._grid._owner = self
        ap = self._agent_pos
        assert (ap >= (0, 0) if isinstance(ap, tuple) else all(np.asarray(ap) >= 0)) and self._agent_dir >= 0
        start_cell = self._grid.get(*ap)
        assert start_cell is None or start_cell.can_overlap()
        self._carrying = None
        self._step_count = 0
        self._push_pending = True
        return self._grid.encode(), (int(ap[0]), int(ap[1]), int(self._agent_dir))

    def step(self, action):
        self._sync_to_device()
        d = self._dev
        try:
            a = int(action)
            if a != action:
                a = -1
        except (TypeError, ValueError):
            a = -1
        d.act[0] = a
        rc = d.L.mgdp_envs_step(d.h, _lib.ptr(d.act), _lib.ptr(d.obs), _lib.ptr(d.dir), _lib.ptr(d.rew),
                                _lib.ptr(d.term), _lib.ptr(d.trunc), _lib.ptr(d.status))
        self._host_stale = True
        if rc == _lib.MGDP_E_ACTION:
            raise ValueError(f"Unknown action: {action}")
        _lib.check(rc, "mgdp_envs_step")
        terminated = bool(d.term[0])
        truncated = bool(d.trunc[0])
        reward = float(d.rew[0]) if d.rew[0] != 0.0 else 0
        obs = {"image": d.obs[0].copy(), "direction": int(d.dir[0]), "mission": self.mission}
        return obs, reward, terminated, truncated, {}

    def gen_obs(self):
        self._sync_to_device()
        d = self._dev
        _lib.check(d.L.mgdp_envs_observe(d.h, _lib.ptr(d.obs), _lib.ptr(d.dir)), "mgdp_envs_observe")
        return {"image": d.obs[0].copy(), "direction": int(d.dir[0]), "mission": self.mission}

    # ------------------------------------------------------------------ reference helpers
    def _reward(self) -> float:
        return 1 - 0.9 * (self.step_count / self.max_steps)

    @property
    def steps_remaining(self):
        return self.max_steps - self.step_count

    @abstractmethod
    def _gen_grid(self, width, height):
        pass

    def _rand_int(self, low: int, high: int) -> int:
        return self.np_random.integers(low, high)

    def _rand_float(self, low: float, high: float) -> float:
        return self.np_random.uniform(low, high)

    def _rand_bool(self) -> bool:
        return self.np_random.integers(0, 2) == 0

    def _rand_elem(self, iterable: Iterable[T]) -> T:
        lst = list(iterable)
        idx = self._rand_int(0, len(lst))
        return lst[idx]

    def _rand_subset(self, iterable: Iterable[T], num_elems: int) -> list[T]:
        lst = list(iterable)
        assert num_elems <= len(lst)
        out: list[T] = []
        while len(out) < num_elems:
            elem = self._rand_elem(lst)
            lst.remove(elem)
            out.append(elem)
        return out

    def _rand_color(self) -> str:
        return self._rand_elem(COLOR_NAMES)

    def _rand_pos(self, x_low, x_high, y_low, y_high):
        return (self.np_random.integers(x_low, x_high), self.np_random.integers(y_low, y_high))

    def place_obj(self, obj: WorldObj | None, top=None, size=None, reject_fn=None, max_tries=math.inf):
        """Rejection-sample an empty cell (minigrid_env.py:308-367), same RNG call order."""
        if top is None:
            top = (0, 0)
        else:
            top = (max(top[0], 0), max(top[1], 0))
        if size is None:
            size = (self._grid.width, self._grid.height)
        num_tries = 0
        g = self._grid
        while True:
            if num_tries > max_tries:
                raise RecursionError("rejection sampling failed in place_obj")
            num_tries += 1
            pos = (
                self._rand_int(top[0], min(top[0] + size[0], g.width)),
                self._rand_int(top[1], min(top[1] + size[1], g.height)),
            )
            if not g.is_empty(*pos):
                continue
            if np.array_equal(pos, self._agent_pos):
                continue
            if reject_fn and reject_fn(self, pos):
                continue
            break
        g.set(pos[0], pos[1], obj)
        if obj is not None:
            obj.init_pos = pos
            obj.cur_pos = pos
        return pos

    def put_obj(self, obj: WorldObj, i: int, j: int):
        self._grid.set(i, j, obj)
        obj.init_pos = (i, j)
        obj.cur_pos = (i, j)

    def place_agent(self, top=None, size=None, rand_dir=True, max_tries=math.inf):
        self._agent_pos = (-1, -1)
        pos = self.place_obj(None, top, size, max_tries=max_tries)
        self._agent_pos = pos
        if rand_dir:
            self._agent_dir = self._rand_int(0, 4)
        return pos

    @property
    def dir_vec(self):
        d = self.agent_dir
        assert 0 <= d < 4, f"Invalid agent_dir: {d} is not within range(0, 4)"
        return DIR_TO_VEC[d]

    @property
    def right_vec(self):
        dx, dy = self.dir_vec
        return np.array((-dy, dx))

    @property
    def front_pos(self):
        return self.agent_pos + self.dir_vec

    def get_view_coords(self, i, j):
        ax, ay = self.agent_pos
        dx, dy = self.dir_vec
        rx, ry = self.right_vec
        sz = self.agent_view_size
        hs = self.agent_view_size // 2
        tx = ax + (dx * (sz - 1)) - (rx * hs)
        ty = ay + (dy * (sz - 1)) - (ry * hs)
        lx = i - tx
        ly = j - ty
        vx = rx * lx + ry * ly
        vy = -(dx * lx + dy * ly)
        return vx, vy

    def relative_coords(self, x, y):
        vx, vy = self.get_view_coords(x, y)
        if vx < 0 or vy < 0 or vx >= self.agent_view_size or vy >= self.agent_view_size:
            return None
        return vx, vy

    def in_view(self, x, y):
        return self.relative_coords(x, y) is not None

    def agent_sees(self, x, y):
        coordinates = self.relative_coords(x, y)
        if coordinates is None:
            return False
        vx, vy = coordinates
        obs = self.gen_obs()
        obs_grid, _ = Grid.decode(obs["image"])
        obs_cell = obs_grid.get(vx, vy)
        world_cell = self.grid.get(x, y)
        assert world_cell is not None
        return obs_cell is not None and obs_cell.type == world_cell.type

    def pprint_grid(self):
        if self._agent_pos is None or self._agent_dir is None or self._grid is None:
            raise ValueError("The environment hasn't been `reset` therefore the `agent_pos`, "
                             "`agent_dir` or `grid` are unknown.")
        short = {"wall": "W", "floor": "F", "door": "D", "key": "K", "ball": "A", "box": "B",
                 "goal": "G", "lava": "V"}
        arrows = {0: ">", 1: "V", 2: "<", 3: "^"}
        g, (ax, ay), ad = self.grid, self.agent_pos, self.agent_dir
        out = ""
        for j in range(g.height):
            for i in range(g.width):
                if i == ax and j == ay:
                    out += 2 * arrows[ad]
                    continue
                tile = g.get(i, j)
                if tile is None:
                    out += "  "
                elif tile.type == "door":
                    out += "__" if tile.is_open else ("L" if tile.is_locked else "D") + tile.color[0].upper()
                else:
                    out += short[tile.type] + tile.color[0].upper()
            if j < g.height - 1:
                out += "\n"
        return out

    def cells(self) -> np.ndarray:
        """(H, W) OBJECT_TO_IDX codes of the current grid: the value-iteration input."""
        return self.grid.cells()

    def render(self):
        raise NotImplementedError("rendering is outside this engine's scope (DESIGN.md)")

    def close(self):
        self._dev = None

    def __getstate__(self):
        self._pull()
        d = dict(self.__dict__)
        d["_dev"] = None
        d["_push_pending"] = True
        d["_host_stale"] = False
        return d

    def __setstate__(self, d):
        self.__dict__.update(d)
        self._grid._owner = self
