"""Empty stand-in: minigrid imports pygame at module level for rendering, which is out of scope."""
