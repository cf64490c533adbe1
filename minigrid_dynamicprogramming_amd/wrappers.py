"""The two reference wrappers whose semantics the DP models.

Both wrap a MiniGridEnv of this package, whose step() runs on the GPU step kernel:
  StochasticActionWrapper  minigrid/wrappers.py:775-796  -> ValueIteration(slip_p=prob)
  NoDeath                  minigrid/wrappers.py:799-872  -> ValueIteration(lava="nodeath", death_cost=...)
"""
from __future__ import annotations

import numpy as np


class Wrapper:
    """Attribute-forwarding wrapper (gymnasium.Wrapper's role for these two)."""

    def __init__(self, env):
        self.env = env

    def __getattr__(self, name):
        return getattr(self.env, name)

    def reset(self, *, seed=None, options=None):
        return self.env.reset(seed=seed, options=options)

    def step(self, action):
        return self.env.step(action)

    @property
    def unwrapped(self):
        return self.env.unwrapped if hasattr(self.env, "unwrapped") else self.env


class StochasticActionWrapper(Wrapper):
    """With probability 1 - prob the action is replaced by np_random.integers(0, 6) (or a fixed
    random_action); the draw order follows wrappers.py:787-796 (np.random.uniform first)."""

    def __init__(self, env=None, prob=0.9, random_action=None):
        super().__init__(env)
        self.prob = prob
        self.random_action = random_action

    def action(self, action):
        if np.random.uniform() < self.prob:
            return action
        if self.random_action is None:
            return self.np_random.integers(0, high=6)
        return self.random_action

    def step(self, action):
        return self.env.step(self.action(action))


class NoDeath(Wrapper):
    """Entering a cell of a no_death type (lava) gives death_cost instead of ending the episode;
    the agent then stands on it (wrappers.py:799-872)."""

    def __init__(self, env, no_death_types: tuple[str, ...], death_cost: float = -1.0):
        assert "goal" not in no_death_types, "goal cannot be a death cell"
        super().__init__(env)
        self.death_cost = death_cost
        self.no_death_types = no_death_types

    def step(self, action):
        front_cell = self.grid.get(*self.front_pos)
        going_to_death = (action == self.actions.forward and front_cell is not None
                          and front_cell.type in self.no_death_types)
        obs, reward, terminated, truncated, info = self.env.step(action)
        current_cell = self.grid.get(*self.agent_pos)
        in_death = current_cell is not None and current_cell.type in self.no_death_types
        if terminated and (going_to_death or in_death):
            terminated = False
            reward += self.death_cost
        return obs, reward, terminated, truncated, info
