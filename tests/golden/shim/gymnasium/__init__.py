"""Offline stand-in for the slice of the gymnasium API that minigrid 2.3.1 touches.

Test infrastructure only: used by tests/golden/make_golden.py in the build container to import the
reference read-only and capture golden vectors.  It never travels to, or runs on, the GPU box.
Seeding follows gymnasium's published rule: Generator(PCG64(SeedSequence(seed))).
"""
from gymnasium import core, spaces, logger, utils  # noqa: F401
from gymnasium.core import Env, Wrapper, ObservationWrapper, ActionWrapper  # noqa: F401
from gymnasium.utils import seeding  # noqa: F401
