import numpy as np

from gymnasium.utils import seeding


class Space:
    def __init__(self, shape=None, dtype=None, seed=None):
        self.shape = shape
        self.dtype = dtype
        self._np_random = None
        if seed is not None:
            self.seed(seed)

    def __class_getitem__(cls, item):
        return cls

    @property
    def np_random(self):
        if self._np_random is None:
            self.seed()
        return self._np_random

    def seed(self, seed=None):
        self._np_random, s = seeding.np_random(seed)
        return [s]


class Discrete(Space):
    def __init__(self, n, seed=None, start=0):
        self.n = int(n)
        self.start = start
        super().__init__((), np.int64, seed)

    def sample(self):
        return int(self.start + self.np_random.integers(self.n))


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32, seed=None):
        self.low, self.high = low, high
        super().__init__(tuple(shape) if shape is not None else None, np.dtype(dtype), seed)


class MultiDiscrete(Space):
    def __init__(self, nvec, seed=None):
        self.nvec = np.asarray(nvec)
        super().__init__(self.nvec.shape, np.int64, seed)


class Text(Space):
    def __init__(self, max_length, seed=None, **_):
        super().__init__((), str, seed)


class Dict(Space):
    def __init__(self, spaces=None, seed=None, **kw):
        self.spaces = dict(spaces or {}, **kw)
        super().__init__(None, None, seed)

    def __getitem__(self, k):
        return self.spaces[k]
