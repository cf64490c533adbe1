"""Batched reset(seed) grid generation on the GPU (csrc/gen.hip).

generate(env_or_id, seed0, B) returns what B calls of the reference's reset(seed0 + b) produce
(grid encodings, row-major type codes, agent x/y/dir) without the host's per-env Python loop: the
seeding (numpy Generator(PCG64(SeedSequence(seed)))) and each family's _gen_grid run one thread per
env.  Pinned against this package's host generators (themselves pinned to the reference) and the
reference's grid digests (tests/test_gpu_gen.py).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .core import OBJECT_TO_IDX, Lava
from .envs import CrossingEnv, DistShiftEnv, DoorKeyEnv, EmptyEnv, FourRoomsEnv, LavaGapEnv
from .registry import make

GEN_EMPTY, GEN_FOURROOMS, GEN_CROSSING, GEN_DOORKEY, GEN_LAVAGAP, GEN_DISTSHIFT = range(6)


def gen_desc(env) -> _lib.GenDesc:
    """The generator descriptor of an env instance (raises ValueError for unsupported configs)."""
    d = _lib.GenDesc()
    d.W, d.H = env.width, env.height
    if isinstance(env, EmptyEnv):
        d.family = GEN_EMPTY
        if env.agent_start_pos is None:
            d.random_start = 1
        elif tuple(env.agent_start_pos) != (1, 1) or env.agent_start_dir != 0:
            raise ValueError("GPU generation supports EmptyEnv agent_start_pos (1,1) dir 0 or None")
    elif isinstance(env, FourRoomsEnv):
        if env._agent_default_pos is not None or env._goal_default_pos is not None:
            raise ValueError("GPU generation supports FourRooms with random agent and goal")
        d.family = GEN_FOURROOMS
    elif isinstance(env, CrossingEnv):
        d.family = GEN_CROSSING
        d.num_crossings = env.num_crossings
        d.obstacle = OBJECT_TO_IDX["lava"] if env.obstacle_type == Lava else OBJECT_TO_IDX["wall"]
    elif isinstance(env, DoorKeyEnv):
        d.family = GEN_DOORKEY
    elif isinstance(env, LavaGapEnv):
        d.family = GEN_LAVAGAP
        d.obstacle = OBJECT_TO_IDX["lava"] if env.obstacle_type == Lava else OBJECT_TO_IDX["wall"]
    elif isinstance(env, DistShiftEnv):
        if env.agent_start_pos is None or tuple(env.agent_start_pos) != (1, 1) or env.agent_start_dir != 0:
            raise ValueError("GPU generation supports DistShift with the default agent start")
        d.family = GEN_DISTSHIFT
        d.strip2_row = env.strip2_row
    else:
        raise ValueError(f"no GPU generator for {type(env).__name__}")
    return d


def supported(env) -> bool:
    try:
        gen_desc(env)
        return True
    except ValueError:
        return False


def generate(env, seed0: int, B: int, device: int = 0, enc: bool = True, cells: bool = False,
             agent: bool = True) -> dict:
    """Host arrays {"enc": (B, W, H, 3) uint8, "cells": (B, H, W) uint8, "agent": (B, 3) int32}."""
    if isinstance(env, str):
        env = make(env)
    d = gen_desc(env)
    L = _lib.load()
    _lib.require_gpu()
    out = {}
    e = np.empty((B, d.W, d.H, 3), np.uint8) if enc else None
    c = np.empty((B, d.H, d.W), np.uint8) if cells else None
    a = np.empty((B, 3), np.int32) if agent else None
    _lib.check(L.mgdp_gen_grids_host(ctypes.byref(d), int(device), int(seed0), int(B), _lib.ptr(e), _lib.ptr(c),
                                     _lib.ptr(a)), "mgdp_gen_grids_host")
    if enc:
        out["enc"] = e
    if cells:
        out["cells"] = c
    if agent:
        out["agent"] = a
    return out


def generate_device(env, seed0: int, B: int, enc_ptr=None, cells_ptr=None, agent_ptr=None, device: int = 0,
                    stream=None):
    """Asynchronous generation into device buffers (torch CUDA tensors or raw pointers)."""
    if isinstance(env, str):
        env = make(env)
    d = gen_desc(env)
    L = _lib.load()
    _lib.check(L.mgdp_gen_grids(ctypes.byref(d), int(device), ctypes.c_void_p(int(stream) if stream else 0),
                                int(seed0), int(B), _lib.ptr(enc_ptr), _lib.ptr(cells_ptr), _lib.ptr(agent_ptr)),
               "mgdp_gen_grids")
