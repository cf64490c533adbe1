"""Host-side data model: encodings, actions, cell objects and the Grid container.

Mirrors the reference's core layer so that user code reads the same:
  constants    minigrid/core/constants.py:8-58
  Actions      minigrid/core/actions.py:7-20
  WorldObj &c. minigrid/core/world_object.py:27-294 (data + predicates only; no rendering)
  Grid         minigrid/core/grid.py:20-143, 244-289 (no rendering)
The grid is stored as three uint8 planes (type, colour, state), row-major [y][x] -- the same flat
int8 layout that is uploaded to HBM for the HIP kernels -- plus three "held" planes: the object a
Box holds (Box(contains=...), world_object.py:272-294; type 0 = nothing), the HIP step's contents
plane (mgdp_envs_set_contents).
"""
from __future__ import annotations

from enum import IntEnum
from typing import Any, Callable

import numpy as np

# --- encodings (constants.py) -------------------------------------------------------------------
COLORS = {
    "red": np.array([255, 0, 0]),
    "green": np.array([0, 255, 0]),
    "blue": np.array([0, 0, 255]),
    "purple": np.array([112, 39, 195]),
    "yellow": np.array([255, 255, 0]),
    "grey": np.array([100, 100, 100]),
}
COLOR_NAMES = sorted(list(COLORS.keys()))
COLOR_TO_IDX = {"red": 0, "green": 1, "blue": 2, "purple": 3, "yellow": 4, "grey": 5}
IDX_TO_COLOR = dict(zip(COLOR_TO_IDX.values(), COLOR_TO_IDX.keys()))
OBJECT_TO_IDX = {
    "unseen": 0, "empty": 1, "wall": 2, "floor": 3, "door": 4, "key": 5, "ball": 6, "box": 7,
    "goal": 8, "lava": 9, "agent": 10,
}
IDX_TO_OBJECT = dict(zip(OBJECT_TO_IDX.values(), OBJECT_TO_IDX.keys()))
STATE_TO_IDX = {"open": 0, "closed": 1, "locked": 2}
DIR_TO_VEC = [np.array((1, 0)), np.array((0, 1)), np.array((-1, 0)), np.array((0, -1))]
TILE_PIXELS = 32


class Actions(IntEnum):
    left = 0
    right = 1
    forward = 2
    pickup = 3
    drop = 4
    toggle = 5
    done = 6


# --- cell objects (world_object.py) -------------------------------------------------------------
class WorldObj:
    def __init__(self, type: str, color: str):
        assert type in OBJECT_TO_IDX, type
        assert color in COLOR_TO_IDX, color
        self.type = type
        self.color = color
        self.contains = None
        self.init_pos = None
        self.cur_pos = None

    def can_overlap(self) -> bool:
        return False

    def can_pickup(self) -> bool:
        return False

    def can_contain(self) -> bool:
        return False

    def see_behind(self) -> bool:
        return True

    def encode(self) -> tuple[int, int, int]:
        return (OBJECT_TO_IDX[self.type], COLOR_TO_IDX[self.color], 0)

    def __repr__(self):
        return f"{type(self).__name__}({self.color!r})"

    @staticmethod
    def decode(type_idx: int, color_idx: int, state: int) -> "WorldObj | None":
        obj_type = IDX_TO_OBJECT[int(type_idx)]
        color = IDX_TO_COLOR[int(color_idx)]
        if obj_type in ("empty", "unseen"):
            return None
        if obj_type == "wall":
            return Wall(color)
        if obj_type == "floor":
            return Floor(color)
        if obj_type == "ball":
            return Ball(color)
        if obj_type == "key":
            return Key(color)
        if obj_type == "box":
            return Box(color)
        if obj_type == "door":
            return Door(color, state == 0, state == 2)
        if obj_type == "goal":
            return Goal()
        if obj_type == "lava":
            return Lava()
        raise AssertionError(f"unknown object type in decode '{obj_type}'")


class Goal(WorldObj):
    def __init__(self):
        super().__init__("goal", "green")

    def can_overlap(self):
        return True


class Floor(WorldObj):
    def __init__(self, color: str = "blue"):
        super().__init__("floor", color)

    def can_overlap(self):
        return True


class Lava(WorldObj):
    def __init__(self):
        super().__init__("lava", "red")

    def can_overlap(self):
        return True


class Wall(WorldObj):
    def __init__(self, color: str = "grey"):
        super().__init__("wall", color)

    def see_behind(self):
        return False


class Door(WorldObj):
    def __init__(self, color: str, is_open: bool = False, is_locked: bool = False):
        super().__init__("door", color)
        self.is_open = is_open
        self.is_locked = is_locked

    def can_overlap(self):
        return self.is_open

    def see_behind(self):
        return self.is_open

    def encode(self):
        state = 0 if self.is_open else (2 if self.is_locked else 1)
        return (OBJECT_TO_IDX[self.type], COLOR_TO_IDX[self.color], state)


class Key(WorldObj):
    def __init__(self, color: str = "blue"):
        super().__init__("key", color)

    def can_pickup(self):
        return True


class Ball(WorldObj):
    def __init__(self, color="blue"):
        super().__init__("ball", color)

    def can_pickup(self):
        return True


class Box(WorldObj):
    """Box (world_object.py:272-294): toggling it puts `contains` in its cell (None: empty), and a
    carried Box keeps what it holds.  One level: a held Box holds nothing (Grid.set refuses more)."""

    def __init__(self, color, contains: WorldObj | None = None):
        super().__init__("box", color)
        self.contains = contains

    def can_pickup(self):
        return True


# --- Grid (grid.py) ------------------------------------------------------------------------------
class Grid:
    """W x H grid as uint8 planes (type, color, state) indexed [y][x].

    get()/set() take (i, j) = (x, y) and assert bounds like the reference (grid.py:65-78).
    An env may bind itself as `owner`; set() then tells the owner to push the grid to the device.
    """

    def __init__(self, width: int, height: int):
        assert width >= 3
        assert height >= 3
        self.width = int(width)
        self.height = int(height)
        self.type = np.full((height, width), OBJECT_TO_IDX["empty"], np.uint8)
        self.color = np.zeros((height, width), np.uint8)
        self.state = np.zeros((height, width), np.uint8)
        # what a Box cell holds: (type, colour, state) planes, type 0 = nothing
        self.held = np.zeros((3, height, width), np.uint8)
        self._owner = None

    # -- element access
    def set(self, i: int, j: int, v: WorldObj | None):
        assert 0 <= i < self.width, f"column index {i} outside of grid of width {self.width}"
        assert 0 <= j < self.height, f"row index {j} outside of grid of height {self.height}"
        held = (0, 0, 0)
        if v is None:
            t, c, s = OBJECT_TO_IDX["empty"], 0, 0
        else:
            inner = getattr(v, "contains", None)
            if inner is not None:
                # the device holds one contents byte per cell (csrc/envs.hip): a Box's object, one level
                if v.type != "box" or getattr(inner, "contains", None) is not None:
                    raise NotImplementedError("only a Box holds an object, and a held Box holds nothing "
                                              "(one contents level; see DESIGN.md)")
                held = inner.encode()
            t, c, s = v.encode()
        self.type[j, i], self.color[j, i], self.state[j, i] = t, c, s
        self.held[:, j, i] = held
        if self._owner is not None:
            self._owner._grid_edited()

    def get(self, i: int, j: int) -> WorldObj | None:
        assert 0 <= i < self.width
        assert 0 <= j < self.height
        v = WorldObj.decode(self.type[j, i], self.color[j, i], self.state[j, i])
        if v is not None and self.held[0, j, i] > OBJECT_TO_IDX["empty"]:
            v.contains = WorldObj.decode(*self.held[:, j, i])
        return v

    def is_empty(self, i: int, j: int) -> bool:
        return self.type[j, i] == OBJECT_TO_IDX["empty"]

    def horz_wall(self, x: int, y: int, length: int | None = None,
                  obj_type: Callable[[], WorldObj] = Wall):
        if length is None:
            length = self.width - x
        for i in range(0, length):
            self.set(x + i, y, obj_type())

    def vert_wall(self, x: int, y: int, length: int | None = None,
                  obj_type: Callable[[], WorldObj] = Wall):
        if length is None:
            length = self.height - y
        for j in range(0, length):
            self.set(x, y + j, obj_type())

    def wall_rect(self, x: int, y: int, w: int, h: int):
        self.horz_wall(x, y, w)
        self.horz_wall(x, y + h - 1, w)
        self.vert_wall(x, y, h)
        self.vert_wall(x + w - 1, y, h)

    # -- encodings
    def encode(self, vis_mask: np.ndarray | None = None) -> np.ndarray:
        """(W, H, 3) uint8, x-major, like grid.py:244-268."""
        arr = np.stack([self.type.T, self.color.T, self.state.T], axis=-1).astype(np.uint8)
        if vis_mask is not None:
            arr = np.where(np.asarray(vis_mask, bool)[:, :, None], arr, 0).astype(np.uint8)
        return arr

    def encode_held(self) -> np.ndarray:
        """(W, H, 3) x-major: what each Box cell holds (zeros elsewhere); mgdp_envs_set_contents' layout."""
        return np.ascontiguousarray(self.held.transpose(2, 1, 0))

    def load_held(self, array: np.ndarray):
        self.held[...] = np.asarray(array, np.uint8).transpose(2, 1, 0)

    @staticmethod
    def decode(array: np.ndarray) -> tuple["Grid", np.ndarray]:
        width, height, channels = array.shape
        assert channels == 3
        g = Grid(width, height)
        g.load_encoding(array)
        vis_mask = array[:, :, 0] != OBJECT_TO_IDX["unseen"]
        return g, vis_mask

    def load_encoding(self, array: np.ndarray):
        a = np.asarray(array, np.uint8)
        t = a[:, :, 0].T.copy()
        t[t == OBJECT_TO_IDX["unseen"]] = OBJECT_TO_IDX["empty"]
        empty = t == OBJECT_TO_IDX["empty"]
        self.type[...] = t
        self.color[...] = np.where(empty, 0, a[:, :, 1].T)
        self.state[...] = np.where(empty, 0, a[:, :, 2].T)
        self.held[...] = 0

    def cells(self) -> np.ndarray:
        """(H, W) OBJECT_TO_IDX codes, row-major: the DP kernels' input layout."""
        return self.type.copy()

    # -- misc (grid.py:37-63)
    def __contains__(self, key: Any) -> bool:
        if isinstance(key, WorldObj):
            key = (key.color, key.type)
        if isinstance(key, tuple):
            color, typ = key
            m = np.ones_like(self.type, bool)
            if typ is not None:
                m &= self.type == OBJECT_TO_IDX[typ]
            else:
                m &= self.type != OBJECT_TO_IDX["empty"]
            if color is not None:
                m &= self.color == COLOR_TO_IDX[color]
            return bool(m.any())
        return False

    def __eq__(self, other) -> bool:
        return isinstance(other, Grid) and np.array_equal(self.encode(), other.encode())

    def __ne__(self, other) -> bool:
        return not self == other

    def copy(self) -> "Grid":
        g = Grid(self.width, self.height)
        g.type[...] = self.type
        g.color[...] = self.color
        g.state[...] = self.state
        g.held[...] = self.held
        return g

    def __getstate__(self):
        d = dict(self.__dict__)
        d["_owner"] = None
        return d
