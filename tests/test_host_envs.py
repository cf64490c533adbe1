"""Host-side grid generation vs the reference (no GPU needed).

reset(seed) -> _gen_grid must reproduce the reference's grid and agent exactly: per-seed encodings
for seeds 0..63 and sha256 digests over the BASELINE batch sizes, all captured from the reference
(tests/golden/make_golden.py).  Also pins the RNG stream via the reference's ReseedWrapper doctest
(minigrid/wrappers.py:27-43).
"""
import hashlib

import numpy as np
import pytest

import minigrid_dynamicprogramming_amd as mg
from tests.golden_util import digests, load

IDS = {
    "empty5": "MiniGrid-Empty-5x5-v0",
    "empty16": "MiniGrid-Empty-16x16-v0",
    "fourrooms": "MiniGrid-FourRooms-v0",
    "lava11n5": "MiniGrid-LavaCrossingS11N5-v0",
    "doorkey16": "MiniGrid-DoorKey-16x16-v0",
    "doorkey8": "MiniGrid-DoorKey-8x8-v0",
    "lavagap5": "MiniGrid-LavaGapS5-v0",
    "lavagap6": "MiniGrid-LavaGapS6-v0",
    "lavagap7": "MiniGrid-LavaGapS7-v0",
    "distshift1": "MiniGrid-DistShift1-v0",
    "distshift2": "MiniGrid-DistShift2-v0",
}


@pytest.mark.parametrize("name", sorted(IDS))
def test_grids_match_reference(name):
    g = load(f"grids_{name}.npz")
    env = mg.make(IDS[name])
    for seed in range(g["enc"].shape[0]):
        enc, agent = env.generate(seed=seed)
        np.testing.assert_array_equal(enc, g["enc"][seed], err_msg=f"{name} seed {seed}")
        assert tuple(agent) == tuple(g["agent"][seed]), f"{name} seed {seed}"


@pytest.mark.parametrize("name,n", [("fourrooms", 4096), ("doorkey16", 65536), ("lava11n5", 65536)])
def test_grid_digests_match_reference(name, n):
    d = digests()[name]
    assert d["seeds"] == n
    env = mg.make(IDS[name])
    h = hashlib.sha256()
    for seed in range(n):
        enc, agent = env.generate(seed=seed)
        h.update(enc.tobytes() + np.array(agent, dtype=np.int32).tobytes())
    assert h.hexdigest() == d["sha256"]


def test_sibling_digest_and_attributes():
    # LavaGap / DistShift, tests/golden/make_golden_f3.py
    import json
    import os

    from tests.golden_util import GOLDEN

    with open(os.path.join(GOLDEN, "digests_f3.json")) as f:
        d = json.load(f)["lavagap7"]
    env = mg.make(IDS["lavagap7"])
    h = hashlib.sha256()
    for seed in range(d["seeds"]):
        enc, agent = env.generate(seed=seed)
        h.update(enc.tobytes() + np.array(agent, dtype=np.int32).tobytes())
    assert h.hexdigest() == d["sha256"]
    for name in ("lavagap5", "lavagap6", "lavagap7", "distshift1", "distshift2"):
        g = load(f"grids_{name}.npz")
        e = mg.make(IDS[name])
        assert e.max_steps == int(g["max_steps"]) and e.see_through_walls == bool(g["see_through"])


def test_rng_stream_doctest():
    # minigrid/wrappers.py:27-29: Empty-5x5 reset(seed=123) then np_random.integers(10) x 10
    env = mg.make("MiniGrid-Empty-5x5-v0")
    env.generate(seed=123)
    assert [int(env.np_random.integers(10)) for _ in range(10)] == [0, 6, 5, 0, 9, 2, 2, 1, 3, 1]


def test_registry_ids_and_kwargs():
    for i in ["MiniGrid-Empty-5x5-v0", "MiniGrid-Empty-16x16-v0", "MiniGrid-FourRooms-v0",
              "MiniGrid-LavaCrossingS11N5-v0", "MiniGrid-DoorKey-16x16-v0", "MiniGrid-SimpleCrossingS9N1-v0"]:
        assert i in mg.registry
    e = mg.make("MiniGrid-Empty-16x16-v0")
    assert (e.width, e.height, e.max_steps, e.see_through_walls) == (16, 16, 1024, True)
    e = mg.make("MiniGrid-FourRooms-v0")
    assert (e.width, e.max_steps, e.see_through_walls) == (19, 100, False)
    e = mg.make("MiniGrid-LavaCrossingS11N5-v0")
    assert (e.width, e.max_steps) == (11, 484)
    e = mg.make("MiniGrid-DoorKey-16x16-v0")
    assert (e.width, e.max_steps) == (16, 2560)
    assert mg.make("MiniGrid-Empty-5x5-v0", max_steps=50).max_steps == 50


def test_grid_api_round_trip():
    env = mg.make("MiniGrid-DoorKey-8x8-v0")
    enc, _ = env.generate(seed=3)
    g, vis = mg.Grid.decode(enc)
    assert vis.all()
    np.testing.assert_array_equal(g.encode(), enc)
    assert ("yellow", "key") in g and ("yellow", "door") in g and ("green", "goal") in g
    assert ("blue", "key") not in g
    door = [g.get(x, y) for x in range(8) for y in range(8) if g.get(x, y) is not None and g.get(x, y).type == "door"][0]
    assert door.is_locked and not door.is_open and door.encode() == (4, 4, 2)
    with pytest.raises(AssertionError):
        g.get(8, 0)


def test_grid_box_contents_on_the_host():
    """Grid keeps what a Box holds (Box(contains=...), world_object.py:272-294) beside its planes:
    encode() is unchanged (a Box encodes as (7, colour, 0)), get() returns the Box with its object,
    copy() keeps it, and more than one level is refused."""
    from minigrid_dynamicprogramming_amd.core import Ball, Box, Grid, Key

    g = Grid(5, 5)
    g.set(1, 2, Box("red", contains=Key("blue")))
    b = g.get(1, 2)
    assert b.type == "box" and b.contains.type == "key" and b.contains.color == "blue"
    assert tuple(g.encode()[1, 2]) == (7, 0, 0)
    assert tuple(g.encode_held()[1, 2]) == (5, 2, 0)
    assert g.copy().get(1, 2).contains.type == "key"
    g.set(1, 2, None)
    assert not g.encode_held().any()
    with pytest.raises(NotImplementedError):
        g.set(2, 2, Box("red", contains=Box("blue", contains=Ball("red"))))
    with pytest.raises(NotImplementedError):
        k = Key("red")
        k.contains = Ball("blue")
        g.set(3, 3, k)
