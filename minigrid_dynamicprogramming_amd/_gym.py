"""gymnasium when importable, else a minimal local stand-in with the same seeding rule.

The reference subclasses gymnasium.Env (minigrid_env.py:24).  gymnasium is not installed in this
image, so the env classes fall back to this module's Env/spaces; seeding is identical to
gymnasium.utils.seeding.np_random: Generator(PCG64(SeedSequence(seed))).
"""
from __future__ import annotations

import numpy as np

try:  # pragma: no cover - exercised only where gymnasium exists
    import gymnasium as _gym
    from gymnasium import spaces  # noqa: F401

    Env = _gym.Env
    HAVE_GYMNASIUM = True
except ImportError:
    HAVE_GYMNASIUM = False

    def np_random(seed=None):
        seq = np.random.SeedSequence(seed)
        return np.random.Generator(np.random.PCG64(seq)), seq.entropy

    class Env:
        _np_random = None
        metadata: dict = {}
        render_mode = None
        spec = None

        def reset(self, *, seed=None, options=None):
            if seed is not None:
                self._np_random, _ = np_random(seed)

        @property
        def np_random(self):
            if self._np_random is None:
                self._np_random, _ = np_random()
            return self._np_random

        @np_random.setter
        def np_random(self, value):
            self._np_random = value

        @property
        def unwrapped(self):
            return self

        def close(self):
            pass

    class _Spaces:
        class Space:
            def __init__(self, shape=None, dtype=None, seed=None):
                self.shape = shape
                self.dtype = dtype
                self._np_random = None
                if seed is not None:
                    self.seed(seed)

            @property
            def np_random(self):
                if self._np_random is None:
                    self.seed()
                return self._np_random

            def seed(self, seed=None):
                self._np_random, s = np_random(seed)
                return [s]

            def contains(self, x):
                return True

            def __contains__(self, x):
                return self.contains(x)

        class Discrete(Space):
            def __init__(self, n, seed=None, start=0):
                self.n = int(n)
                self.start = int(start)
                super().__init__((), np.int64, seed)

            def sample(self):
                return int(self.start + self.np_random.integers(self.n))

            def contains(self, x):
                try:
                    v = int(x)
                except (TypeError, ValueError):
                    return False
                return v == x and self.start <= v < self.start + self.n

        class Box(Space):
            def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
                self.low, self.high = low, high
                super().__init__(tuple(shape) if shape is not None else None, np.dtype(dtype), seed)

            def contains(self, x):
                x = np.asarray(x)
                return x.shape == self.shape and bool(np.all(x >= self.low)) and bool(np.all(x <= self.high))

        class Dict(Space):
            def __init__(self, spaces=None, seed=None, **kw):
                self.spaces = dict(spaces or {}, **kw)
                super().__init__(None, None, seed)

            def __getitem__(self, k):
                return self.spaces[k]

            def contains(self, x):
                return isinstance(x, dict) and all(k in x and s.contains(x[k]) for k, s in self.spaces.items())

    spaces = _Spaces()
