registry = {}


def register(id, entry_point=None, kwargs=None, **_):
    registry[id] = (entry_point, dict(kwargs or {}))
