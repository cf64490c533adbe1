"""The four target env families, with grid generators restated on the host.

Each `_gen_grid` issues the same numpy Generator calls in the same order as the reference, so
reset(seed) yields the reference's grid, agent position and direction exactly (pinned by
tests/test_host_envs.py against grids and sha256 digests captured from the reference).
  EmptyEnv      minigrid/envs/empty.py:68-114
  FourRoomsEnv  minigrid/envs/fourrooms.py:60-128
  CrossingEnv   minigrid/envs/crossing.py:87-184   (LavaCrossing / SimpleCrossing)
  DoorKeyEnv    minigrid/envs/doorkey.py:63-100
and two sibling families with the same cell types, whose grids the XYD DP
model covers unchanged:
  LavaGapEnv    minigrid/envs/lavagap.py:69-136
  DistShiftEnv  minigrid/envs/distshift.py:65-121
"""
from __future__ import annotations

import itertools as itt

import numpy as np

from .core import Door, Goal, Grid, Key, Lava, Wall
from .minigrid_env import MiniGridEnv, MissionSpace


class EmptyEnv(MiniGridEnv):
    def __init__(self, size=8, agent_start_pos=(1, 1), agent_start_dir=0, max_steps: int | None = None, **kwargs):
        self.agent_start_pos = agent_start_pos
        self.agent_start_dir = agent_start_dir
        mission_space = MissionSpace(mission_func=self._gen_mission)
        if max_steps is None:
            max_steps = 4 * size**2
        super().__init__(mission_space=mission_space, grid_size=size, see_through_walls=True,
                         max_steps=max_steps, **kwargs)

    @staticmethod
    def _gen_mission():
        return "get to the green goal square"

    def _gen_grid(self, width, height):
        self.grid = Grid(width, height)
        self.grid.wall_rect(0, 0, width, height)
        self.put_obj(Goal(), width - 2, height - 2)
        if self.agent_start_pos is not None:
            self.agent_pos = self.agent_start_pos
            self.agent_dir = self.agent_start_dir
        else:
            self.place_agent()
        self.mission = "get to the green goal square"


class FourRoomsEnv(MiniGridEnv):
    def __init__(self, agent_pos=None, goal_pos=None, max_steps=100, **kwargs):
        self._agent_default_pos = agent_pos
        self._goal_default_pos = goal_pos
        self.size = 19
        mission_space = MissionSpace(mission_func=self._gen_mission)
        super().__init__(mission_space=mission_space, width=self.size, height=self.size,
                         max_steps=max_steps, **kwargs)

    @staticmethod
    def _gen_mission():
        return "reach the goal"

    def _gen_grid(self, width, height):
        self.grid = Grid(width, height)
        self.grid.horz_wall(0, 0)
        self.grid.horz_wall(0, height - 1)
        self.grid.vert_wall(0, 0)
        self.grid.vert_wall(width - 1, 0)
        room_w = width // 2
        room_h = height // 2
        for j in range(0, 2):
            for i in range(0, 2):
                xL = i * room_w
                yT = j * room_h
                xR = xL + room_w
                yB = yT + room_h
                if i + 1 < 2:
                    self.grid.vert_wall(xR, yT, room_h)
                    pos = (xR, self._rand_int(yT + 1, yB))
                    self.grid.set(*pos, None)
                if j + 1 < 2:
                    self.grid.horz_wall(xL, yB, room_w)
                    pos = (self._rand_int(xL + 1, xR), yB)
                    self.grid.set(*pos, None)
        if self._agent_default_pos is not None:
            self.agent_pos = self._agent_default_pos
            self.grid.set(*self._agent_default_pos, None)
            self.agent_dir = self._rand_int(0, 4)
        else:
            self.place_agent()
        if self._goal_default_pos is not None:
            goal = Goal()
            self.put_obj(goal, *self._goal_default_pos)
            goal.init_pos, goal.cur_pos = self._goal_default_pos
        else:
            self.place_obj(Goal())


class CrossingEnv(MiniGridEnv):
    def __init__(self, size=9, num_crossings=1, obstacle_type=Lava, max_steps: int | None = None, **kwargs):
        self.num_crossings = num_crossings
        self.obstacle_type = obstacle_type
        if obstacle_type == Lava:
            mission_space = MissionSpace(mission_func=self._gen_mission_lava)
        else:
            mission_space = MissionSpace(mission_func=self._gen_mission)
        if max_steps is None:
            max_steps = 4 * size**2
        super().__init__(mission_space=mission_space, grid_size=size, see_through_walls=False,
                         max_steps=max_steps, **kwargs)

    @staticmethod
    def _gen_mission_lava():
        return "avoid the lava and get to the green goal square"

    @staticmethod
    def _gen_mission():
        return "find the opening and get to the green goal square"

    def _gen_grid(self, width, height):
        assert width % 2 == 1 and height % 2 == 1
        self.grid = Grid(width, height)
        self.grid.wall_rect(0, 0, width, height)
        self.agent_pos = np.array((1, 1))
        self.agent_dir = 0
        self.put_obj(Goal(), width - 2, height - 2)
        v, h = object(), object()
        rivers = [(v, i) for i in range(2, height - 2, 2)]
        rivers += [(h, j) for j in range(2, width - 2, 2)]
        self.np_random.shuffle(rivers)
        rivers = rivers[: self.num_crossings]
        rivers_v = sorted(pos for direction, pos in rivers if direction is v)
        rivers_h = sorted(pos for direction, pos in rivers if direction is h)
        obstacle_pos = itt.chain(
            itt.product(range(1, width - 1), rivers_h),
            itt.product(rivers_v, range(1, height - 1)),
        )
        for i, j in obstacle_pos:
            self.put_obj(self.obstacle_type(), i, j)
        path = [h] * len(rivers_v) + [v] * len(rivers_h)
        self.np_random.shuffle(path)
        limits_v = [0] + rivers_v + [height - 1]
        limits_h = [0] + rivers_h + [width - 1]
        room_i, room_j = 0, 0
        for direction in path:
            if direction is h:
                i = limits_v[room_i + 1]
                j = self.np_random.choice(range(limits_h[room_j] + 1, limits_h[room_j + 1]))
                room_i += 1
            elif direction is v:
                i = self.np_random.choice(range(limits_v[room_i] + 1, limits_v[room_i + 1]))
                j = limits_h[room_j + 1]
                room_j += 1
            else:
                raise AssertionError
            self.grid.set(i, j, None)
        self.mission = (
            "avoid the lava and get to the green goal square"
            if self.obstacle_type == Lava
            else "find the opening and get to the green goal square"
        )


class DoorKeyEnv(MiniGridEnv):
    def __init__(self, size=8, max_steps: int | None = None, **kwargs):
        if max_steps is None:
            max_steps = 10 * size**2
        mission_space = MissionSpace(mission_func=self._gen_mission)
        super().__init__(mission_space=mission_space, grid_size=size, max_steps=max_steps, **kwargs)

    @staticmethod
    def _gen_mission():
        return "use the key to open the door and then get to the goal"

    def _gen_grid(self, width, height):
        self.grid = Grid(width, height)
        self.grid.wall_rect(0, 0, width, height)
        self.put_obj(Goal(), width - 2, height - 2)
        splitIdx = self._rand_int(2, width - 2)
        self.grid.vert_wall(splitIdx, 0)
        self.place_agent(size=(splitIdx, height))
        doorIdx = self._rand_int(1, width - 2)
        self.put_obj(Door("yellow", is_locked=True), splitIdx, doorIdx)
        self.place_obj(obj=Key("yellow"), top=(0, 0), size=(splitIdx, height))
        self.mission = "use the key to open the door and then get to the goal"


class LavaGapEnv(MiniGridEnv):
    """A vertical strip of lava (or walls) with one gap between the agent at (1,1) and the goal at
    (W-2, H-2); lavagap.py:69-136."""

    def __init__(self, size, obstacle_type=Lava, max_steps: int | None = None, **kwargs):
        self.obstacle_type = obstacle_type
        self.size = size
        mission_space = MissionSpace(mission_func=self._gen_mission_lava if obstacle_type == Lava
                                     else self._gen_mission)
        if max_steps is None:
            max_steps = 4 * size**2
        super().__init__(mission_space=mission_space, width=size, height=size, see_through_walls=False,
                         max_steps=max_steps, **kwargs)

    @staticmethod
    def _gen_mission_lava():
        return "avoid the lava and get to the green goal square"

    @staticmethod
    def _gen_mission():
        return "find the opening and get to the green goal square"

    def _gen_grid(self, width, height):
        assert width >= 5 and height >= 5
        self.grid = Grid(width, height)
        self.grid.wall_rect(0, 0, width, height)
        self.agent_pos = np.array((1, 1))
        self.agent_dir = 0
        self.goal_pos = np.array((width - 2, height - 2))
        self.put_obj(Goal(), *self.goal_pos)
        # the gap: one random column in [2, W-2), one random row in [1, H-1), in that draw order
        self.gap_pos = np.array((self._rand_int(2, width - 2), self._rand_int(1, height - 1)))
        self.grid.vert_wall(self.gap_pos[0], 1, height - 2, self.obstacle_type)
        self.grid.set(*self.gap_pos, None)
        self.mission = ("avoid the lava and get to the green goal square" if self.obstacle_type == Lava
                        else "find the opening and get to the green goal square")


class DistShiftEnv(MiniGridEnv):
    """Two lava strips between the agent and the goal at (W-2, 1); the second strip's row is the
    distributional-shift knob; distshift.py:65-121."""

    def __init__(self, width=9, height=7, agent_start_pos=(1, 1), agent_start_dir=0, strip2_row=2,
                 max_steps: int | None = None, **kwargs):
        self.agent_start_pos = agent_start_pos
        self.agent_start_dir = agent_start_dir
        self.goal_pos = (width - 2, 1)
        self.strip2_row = strip2_row
        mission_space = MissionSpace(mission_func=self._gen_mission)
        if max_steps is None:
            max_steps = 4 * width * height
        super().__init__(mission_space=mission_space, width=width, height=height, see_through_walls=True,
                         max_steps=max_steps, **kwargs)

    @staticmethod
    def _gen_mission():
        return "get to the green goal square"

    def _gen_grid(self, width, height):
        self.grid = Grid(width, height)
        self.grid.wall_rect(0, 0, width, height)
        self.put_obj(Goal(), *self.goal_pos)
        for i in range(self.width - 6):
            self.grid.set(3 + i, 1, Lava())
            self.grid.set(3 + i, self.strip2_row, Lava())
        if self.agent_start_pos is not None:
            self.agent_pos = self.agent_start_pos
            self.agent_dir = self.agent_start_dir
        else:
            self.place_agent()
        self.mission = "get to the green goal square"


__all__ = ["EmptyEnv", "FourRoomsEnv", "CrossingEnv", "DoorKeyEnv", "LavaGapEnv", "DistShiftEnv", "Wall", "Lava"]
