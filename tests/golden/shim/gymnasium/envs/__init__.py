from gymnasium.envs import registration  # noqa: F401
