"""Batched MiniGrid stepping on one GPU: B envs resident in HBM, one HIP launch per step.

The reference vectorises with gymnasium's in-process SyncVectorEnv (tests/test_envs.py:310-330),
which loops MiniGridEnv.step (minigrid_env.py:520-590) serially.  Here every env's grid planes and
agent state live in HBM and one envs_step_kernel launch advances all of them (csrc/envs.hip).
Grids are generated on the host by the reference-exact generators (envs.py) and uploaded on reset.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib, gen
from .registry import make


class MiniGridVecEnv:
    """B independent envs of one registered id (same W, H), stepped together on one GPU.

    step(actions) -> (obs, reward, terminated, truncated, info) with obs = {"image": (B,V,V,3) uint8,
    "direction": (B,) int32, "mission": [str]*B}.  autoreset=True resets finished envs right after
    the step with their next seed (the returned obs is then the reset observation and the final
    observation is in info["final_obs_image"]).
    """

    def __init__(self, env_id: str, num_envs: int, device: int = 0, autoreset: bool = False,
                 no_death_types: tuple = (), death_cost: float = -1.0, **kwargs):
        """no_death_types / death_cost: NoDeath(env, no_death_types, death_cost) applied inside the
        step kernel (wrappers.py:799-872)."""
        self.env_id = env_id
        self.num_envs = int(num_envs)
        self.autoreset = autoreset
        self._gen = make(env_id, **kwargs)  # host-side generator (one instance reused per seed)
        self._gpu_gen = gen.supported(self._gen)  # reset(seed) batches generated on the GPU
        self.device = device
        self.W, self.H = self._gen.width, self._gen.height
        self.view = self._gen.agent_view_size
        self.max_steps = self._gen.max_steps
        self.see_through = self._gen.see_through_walls
        self.mission = self._gen.mission
        self.L = _lib.load()
        _lib.require_gpu()
        h = ctypes.c_void_p()
        _lib.check(self.L.mgdp_envs_create(device, self.num_envs, self.W, self.H, self.view, ctypes.byref(h)),
                   "mgdp_envs_create")
        self.h = h
        if no_death_types:
            assert "goal" not in no_death_types, "goal cannot be a death cell"
            from .core import OBJECT_TO_IDX

            mask = 0
            for t in no_death_types:
                mask |= 1 << OBJECT_TO_IDX[t]
            _lib.check(self.L.mgdp_envs_set_nodeath(h, mask, float(death_cost)), "mgdp_envs_set_nodeath")
        B, V = self.num_envs, self.view
        self._obs = np.zeros((B, V, V, 3), np.uint8)
        self._dir = np.zeros(B, np.int32)
        self._rew = np.zeros(B, np.float64)
        self._term = np.zeros(B, np.uint8)
        self._trunc = np.zeros(B, np.uint8)
        self._status = np.zeros(B, np.int32)
        self._seeds = np.zeros(B, np.int64)
        self._next_seed = 0
        self._held = False  # Box contents planes in use (set_contents)

    def close(self):
        if getattr(self, "h", None):
            self.L.mgdp_envs_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- raw state upload
    def load(self, enc: np.ndarray, agent: np.ndarray, max_steps=None, see_through=None, mask=None, held=None):
        """Upload grids (B, W, H, 3) x-major encodings and agents (B, 3) = (x, y, dir).  held: what
        each Box cell holds (Box(contains=...)), the same layout, type 0 = nothing (set_contents)."""
        B = self.num_envs
        enc = np.ascontiguousarray(enc, np.uint8)
        agent = np.ascontiguousarray(agent, np.int32)
        assert enc.shape == (B, self.W, self.H, 3) and agent.shape == (B, 3)
        ms = np.full(B, self.max_steps if max_steps is None else 0, np.int32)
        if max_steps is not None:
            ms[:] = np.asarray(max_steps, np.int32)
        see = np.full(B, 1 if self.see_through else 0, np.uint8)
        if see_through is not None:
            see[:] = np.asarray(see_through, np.uint8)
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        _lib.check(self.L.mgdp_envs_load(self.h, _lib.ptr(enc), _lib.ptr(agent), _lib.ptr(ms), _lib.ptr(see),
                                         _lib.ptr(m)), "mgdp_envs_load")
        if held is not None:
            if mask is not None:  # the other envs keep theirs
                cur = self.get_contents()[0]
                sel = np.asarray(mask, bool)
                cur[sel] = np.asarray(held, np.uint8)[sel]
                held = cur
            self.set_contents(held)

    def set_contents(self, held=None, carry_held=None):
        """Box(contains=...) (world_object.py:272-294): held (B, W, H, 3) = the (type, colour, state)
        each Box cell holds, carry_held (B, 3) = what a carried Box holds (None = unchanged).  Toggling
        a Box then puts its object in the cell, and a carried Box keeps it (mgdp_envs_set_contents)."""
        B = self.num_envs
        h = None if held is None else np.ascontiguousarray(held, np.uint8)
        c = None if carry_held is None else np.ascontiguousarray(carry_held, np.int32)
        assert h is None or h.shape == (B, self.W, self.H, 3)
        assert c is None or c.shape == (B, 3)
        _lib.check(self.L.mgdp_envs_set_contents(self.h, _lib.ptr(h), _lib.ptr(c)), "mgdp_envs_set_contents")
        self._held = True

    def get_contents(self):
        """(held (B, W, H, 3), carry_held (B, 3)): what the Boxes hold now (zeros: nothing)."""
        B = self.num_envs
        held = np.zeros((B, self.W, self.H, 3), np.uint8)
        carry_held = np.zeros((B, 3), np.int32)
        _lib.check(self.L.mgdp_envs_get_contents(self.h, _lib.ptr(held), _lib.ptr(carry_held)),
                   "mgdp_envs_get_contents")
        return held, carry_held

    def _generate(self, seeds):
        seeds = np.asarray(seeds, np.int64)
        if self._gpu_gen and len(seeds) and (np.diff(seeds) == 1).all():
            # consecutive seeds: one generator launch (csrc/gen.hip) instead of a host loop
            out = gen.generate(self._gen, int(seeds[0]), len(seeds), device=self.device)
            return out["enc"], out["agent"]
        encs, agents = [], []
        for s in seeds:
            e, a = self._gen.generate(seed=int(s))
            encs.append(e)
            agents.append(a)
        return np.stack(encs), np.array(agents, np.int32)

    def observe(self):
        _lib.check(self.L.mgdp_envs_observe(self.h, _lib.ptr(self._obs), _lib.ptr(self._dir)), "mgdp_envs_observe")
        return self._obs_dict()

    def _obs_dict(self):
        return {"image": self._obs.copy(), "direction": self._dir.copy(), "mission": [self.mission] * self.num_envs}

    # ---------------------------------------------------------------- gym-style API
    def reset(self, seed: int | None = None):
        if seed is None:
            seed = int(np.random.SeedSequence().generate_state(1)[0])
        self._seeds = np.arange(self.num_envs, dtype=np.int64) + int(seed)
        self._next_seed = int(seed) + self.num_envs
        enc, agent = self._generate(self._seeds)
        self.load(enc, agent)
        return self.observe(), {"seeds": self._seeds.copy()}

    def step(self, actions):
        a = np.ascontiguousarray(np.asarray(actions).reshape(self.num_envs), np.int32)
        rc = self.L.mgdp_envs_step(self.h, _lib.ptr(a), _lib.ptr(self._obs), _lib.ptr(self._dir),
                                   _lib.ptr(self._rew), _lib.ptr(self._term), _lib.ptr(self._trunc),
                                   _lib.ptr(self._status))
        if rc == _lib.MGDP_E_ACTION:
            bad = np.flatnonzero(self._status == _lib.MGDP_E_ACTION)
            raise ValueError(f"Unknown action: {actions[bad[0]] if len(bad) else actions} (env {bad.tolist()})")
        _lib.check(rc, "mgdp_envs_step")
        obs = self._obs_dict()
        term = self._term.astype(bool)
        trunc = self._trunc.astype(bool)
        info = {}
        if self.autoreset:
            done = term | trunc
            if done.any():
                info["final_obs_image"] = obs["image"].copy()
                idx = np.flatnonzero(done)
                seeds = self._next_seed + np.arange(len(idx))
                self._next_seed += len(idx)
                self._seeds[idx] = seeds
                enc = np.zeros((self.num_envs, self.W, self.H, 3), np.uint8)
                agent = np.zeros((self.num_envs, 3), np.int32)
                e, ag = self._generate(seeds)
                enc[idx], agent[idx] = e, ag
                mask = done.astype(np.uint8)
                self.load(enc, agent, mask=mask)
                obs = self.observe()
        return obs, self._rew.copy(), term, trunc, info

    def step_device(self, actions, obs, direction, reward, terminated, truncated, status):
        """Zero-copy step on device buffers (torch CUDA tensors or raw device pointers as ints),
        asynchronous on the handle's stream.  Raw pointers skip every per-call conversion."""
        p = _lib.ptr
        rc = self.L.mgdp_envs_step_device(self.h, p(actions), p(obs), p(direction), p(reward), p(terminated),
                                          p(truncated), p(status))
        if rc:
            _lib.check(rc, "mgdp_envs_step_device")

    def enable_timing(self, on: bool):
        """Time every step-kernel launch with a HIP event pair on the launch itself."""
        _lib.check(self.L.mgdp_envs_enable_timing(self.h, int(on)), "mgdp_envs_enable_timing")

    def kernel_time(self):
        """(total ms, launches) of the step kernel since enable_timing(True); synchronises."""
        ms, n = ctypes.c_double(0), ctypes.c_int64(0)
        _lib.check(self.L.mgdp_envs_kernel_time(self.h, ctypes.byref(ms), ctypes.byref(n)), "mgdp_envs_kernel_time")
        return ms.value, n.value

    def set_stream(self, stream):
        _lib.check(self.L.mgdp_envs_set_stream(self.h, ctypes.c_void_p(int(stream) if stream else 0)),
                   "mgdp_envs_set_stream")

    def get_state(self):
        B = self.num_envs
        enc = np.zeros((B, self.W, self.H, 3), np.uint8)
        agent = np.zeros((B, 3), np.int32)
        carry = np.zeros((B, 2), np.int32)
        sc = np.zeros(B, np.int32)
        _lib.check(self.L.mgdp_envs_get_state(self.h, _lib.ptr(enc), _lib.ptr(agent), _lib.ptr(carry), _lib.ptr(sc)),
                   "mgdp_envs_get_state")
        st = {"enc": enc, "agent": agent, "carry": carry, "step_count": sc}
        if self._held:
            st["held"], st["carry_held"] = self.get_contents()
        return st
