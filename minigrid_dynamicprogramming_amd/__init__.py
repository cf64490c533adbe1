"""MI355X-native Minigrid step + tabular value-iteration engine.

Hot path (HIP, gfx950, libmgdp.so behind include/mgdp.h):
  * MiniGridEnv.step / gen_obs for batches of envs            (csrc/envs.hip)
  * Jacobi value iteration over (pos, dir[, has_key, door_open]) (csrc/vi.hip)
Host side (this package): the reference's env API, registry and grid generators, the DP front end
and the multi-GPU driver.  See DESIGN.md.
"""
from .core import (COLOR_NAMES, COLOR_TO_IDX, DIR_TO_VEC, IDX_TO_COLOR, IDX_TO_OBJECT, OBJECT_TO_IDX,
                   STATE_TO_IDX, Actions, Ball, Box, Door, Floor, Goal, Grid, Key, Lava, Wall, WorldObj)
from .minigrid_env import MiniGridEnv, MissionSpace
from .envs import CrossingEnv, DistShiftEnv, DoorKeyEnv, EmptyEnv, FourRoomsEnv, LavaGapEnv
from .registry import EnvSpec, make, register, registry
from .dp import ValueIteration, VIResult, value_iteration
from .vector import MiniGridVecEnv

__version__ = "0.1.0"
