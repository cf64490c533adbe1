from gymnasium.utils import seeding  # noqa: F401
