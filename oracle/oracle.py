"""ctypes front end of the CPU oracle (oracle/mgdp_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, always as the checker, never as the thing measured or shipped.  The product package
minigrid_dynamicprogramming_amd/ must not import this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# MGDP_ORACLE_LIB: an alternative build of the same source (the sanitizer build, oracle/Makefile asan)
LIB_PATH = os.environ.get("MGDP_ORACLE_LIB") or os.path.join(HERE, "libmgdp_oracle.so")

_lib = None

_P = ctypes.c_void_p
_I = ctypes.c_int
_D = ctypes.c_double


def build() -> str:
    """Compile the oracle library in place (gcc; no GPU needed)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.orc_build_table.argtypes = [_I, _I, _I, _P, _P, _P, _P]
        L.orc_vi.argtypes = [_I, _I, _I, _I, _I, _P, _D, _D, _D, _I, _I, _P, _P, _P, _P, _P]
        L.orc_vi_fp.argtypes = [_I, _I, _I, _I, _I, _P, _D, _D, _D, _I, _I, _P, _P, _P, _P, _P, _P]
        L.orc_step.argtypes = [_I, _I, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P]
        L.orc_gen_obs.argtypes = [_I, _I, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P]
        L.orc_vi_ex.argtypes = [_I, _I, _I, _I, _I, _P, _D, _D, _D, _I, _I, _I, _D, _I, _P, _P, _P, _P, _P]
        L.orc_xyd_next_nodeath.argtypes = [_P, _I, _I, _I, _I, _D, _P, _P, _P]
        L.orc_reward.argtypes = [_I, _I]
        L.orc_step_batch.argtypes = [_I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P, _I]
        L.orc_step_batch.restype = None
        L.orc_step_held.argtypes = [_I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P]
        L.orc_step_batch_held.argtypes = [_I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P,
                                          _P, _P, _P, _P, _I]
        L.orc_step_batch_held.restype = None
        L.orc_reward.restype = _D
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def n_actions(model: int) -> int:
    return 7 if model == 0 else 5


def n_states(model: int, W: int, H: int) -> int:
    return W * H * (4 if model == 0 else 16)


def build_table(model: int, cells: np.ndarray):
    """cells: (H, W) uint8 OBJECT_TO_IDX codes, row-major.  Returns nxt, rew, done (S x A)."""
    cells = np.ascontiguousarray(cells, dtype=np.uint8)
    H, W = cells.shape
    S, A = n_states(model, W, H), n_actions(model)
    nxt = np.empty((S, A), np.int32)
    rew = np.empty((S, A), np.float64)
    done = np.empty((S, A), np.uint8)
    lib().orc_build_table(model, W, H, _ptr(cells), _ptr(nxt), _ptr(rew), _ptr(done))
    return nxt, rew, done


def value_iteration(model: int, cells: np.ndarray, gamma=0.99, tol=1e-6, slip_p=None,
                    max_sweeps=10000, dtype="f64", nthreads=1, fixed_point=False):
    """cells: (B, H, W) or (H, W) uint8.  Returns dict(V (B,S), pi (B,S), sweeps, dv_trace, dv).
    fixed_point: orc_vi_fp -- a grid at an exact fixed point is not swept again (same V, pi, sweeps
    and dv as the literal loop); the dict then also holds grid_sweeps (B,), the sweeps each grid ran."""
    cells = np.ascontiguousarray(cells, dtype=np.uint8)
    if cells.ndim == 2:
        cells = cells[None]
    B, H, W = cells.shape
    S = n_states(model, W, H)
    npdt = np.float32 if dtype == "f32" else np.float64
    V = np.empty((B, S), npdt)
    pi = np.empty((B, S), np.int8)
    sweeps = ctypes.c_int(0)
    dv_last = ctypes.c_double(0)
    trace = np.zeros(max_sweeps, np.float64)
    args = (model, 0 if dtype == "f32" else 1, B, W, H, _ptr(cells), gamma, tol,
            -1.0 if slip_p is None else float(slip_p), max_sweeps, nthreads, _ptr(V),
            _ptr(pi), ctypes.byref(sweeps), _ptr(trace), ctypes.byref(dv_last))
    gs = np.zeros(B, np.int32) if fixed_point else None
    rc = lib().orc_vi_fp(*args, _ptr(gs)) if fixed_point else lib().orc_vi(*args)
    if rc != 0:
        raise ValueError(f"orc_vi failed rc={rc}")
    k = sweeps.value
    out = {"V": V, "pi": pi, "sweeps": k, "dv_trace": trace[:k].copy(), "dv": dv_last.value}
    if gs is not None:
        out["grid_sweeps"] = gs
    return out


def value_iteration_ex(model: int, cells: np.ndarray, gamma=0.99, tol=1e-6, slip_p=None,
                       max_sweeps=10000, dtype="f64", nthreads=1, lava_mode=0, death_cost=-1.0,
                       horizon=0, keep_policy_t=False):
    """orc_vi_ex: value_iteration plus NoDeath lava (lava_mode=1) and the finite-horizon DP with the
    exact _reward() (horizon = max_steps > 0).  Returns dict(V, pi, sweeps, dv[, pi_t (H,B,S)])."""
    cells = np.ascontiguousarray(cells, dtype=np.uint8)
    if cells.ndim == 2:
        cells = cells[None]
    B, H, W = cells.shape
    S = n_states(model, W, H)
    npdt = np.float32 if dtype == "f32" else np.float64
    V = np.empty((B, S), npdt)
    pi = np.empty((B, S), np.int8)
    pi_t = np.empty((horizon, B, S), np.int8) if (horizon > 0 and keep_policy_t) else None
    sweeps = ctypes.c_int(0)
    dv_last = ctypes.c_double(0)
    rc = lib().orc_vi_ex(model, 0 if dtype == "f32" else 1, B, W, H, _ptr(cells), gamma, tol,
                         -1.0 if slip_p is None else float(slip_p), max_sweeps, nthreads, int(lava_mode),
                         float(death_cost), int(horizon), _ptr(V), _ptr(pi), _ptr(pi_t),
                         ctypes.byref(sweeps), ctypes.byref(dv_last))
    if rc != 0:
        raise ValueError(f"orc_vi_ex failed rc={rc}")
    out = {"V": V, "pi": pi, "sweeps": sweeps.value, "dv": dv_last.value}
    if pi_t is not None:
        out["pi_t"] = pi_t
    return out


def reward(step_count: int, max_steps: int) -> float:
    return lib().orc_reward(step_count, max_steps)


def gen_obs(planes, agent, carry=(0, 0), see_through=False, view=7):
    """planes: (3, H, W) uint8 (type, color, state).  agent = (x, y, dir)."""
    ty, co, st = (np.ascontiguousarray(p, dtype=np.uint8) for p in planes)
    H, W = ty.shape
    img = np.zeros((view, view, 3), np.uint8)
    lib().orc_gen_obs(W, H, _ptr(ty), _ptr(co), _ptr(st), int(agent[0]), int(agent[1]),
                      int(agent[2]), int(carry[0]), int(carry[1]), int(see_through), view, _ptr(img))
    return img


class OracleBatch:
    """B envs in the GPU engine's layout (row-major planes [B][HWp], agent [B][4]) stepped by the
    oracle's MiniGridEnv.step restatement (orc_step_batch); the step path's CPU baseline."""

    def __init__(self, enc: np.ndarray, agent: np.ndarray, max_steps, see_through, view=7, held=None):
        """held: optional (B, W, H, 3) encodings of what each Box cell holds (type 0 = nothing)."""
        enc = np.asarray(enc, np.uint8)  # (B, W, H, 3) x-major encodings
        B, W, H, _ = enc.shape
        self.B, self.W, self.H, self.view = B, W, H, view
        self.HWp = (W * H + 15) // 16 * 16

        def planes_of(e):
            planes = np.zeros((3, B, self.HWp), np.uint8)
            for p in range(3):
                planes[p, :, : W * H] = e[..., p].transpose(0, 2, 1).reshape(B, W * H)
            return tuple(np.ascontiguousarray(planes[p]) for p in range(3))

        self.ty, self.co, self.st = planes_of(enc)
        self.hty = self.hco = self.hst = None
        self.held_carry = np.zeros((B, 3), np.int32)
        if held is not None:
            self.hty, self.hco, self.hst = planes_of(np.asarray(held, np.uint8))
        self.state = np.zeros((B, 4), np.int32)
        self.state[:, :3] = np.asarray(agent, np.int32)[:, :3]
        self.carry = np.zeros((B, 2), np.int32)
        self.max_steps = np.broadcast_to(np.asarray(max_steps, np.int32), (B,)).copy()
        self.see = np.broadcast_to(np.asarray(see_through, np.uint8), (B,)).copy()
        self.obs = np.zeros((B, view, view, 3), np.uint8)
        self.reward = np.zeros(B, np.float64)
        self.terminated = np.zeros(B, np.uint8)
        self.truncated = np.zeros(B, np.uint8)
        self.status = np.zeros(B, np.int32)

    def step(self, actions: np.ndarray, nthreads: int = 1):
        a = np.ascontiguousarray(actions, np.int32)
        if self.hty is not None:
            lib().orc_step_batch_held(self.B, self.W, self.H, self.HWp, _ptr(self.ty), _ptr(self.co), _ptr(self.st),
                                      _ptr(self.hty), _ptr(self.hco), _ptr(self.hst), _ptr(self.held_carry),
                                      _ptr(self.state), _ptr(self.carry), _ptr(self.max_steps), _ptr(self.see),
                                      self.view, _ptr(a), _ptr(self.obs), _ptr(self.reward), _ptr(self.terminated),
                                      _ptr(self.truncated), _ptr(self.status), int(nthreads))
            return
        lib().orc_step_batch(self.B, self.W, self.H, self.HWp, _ptr(self.ty), _ptr(self.co), _ptr(self.st),
                             _ptr(self.state), _ptr(self.carry), _ptr(self.max_steps), _ptr(self.see), self.view,
                             _ptr(a), _ptr(self.obs), _ptr(self.reward), _ptr(self.terminated),
                             _ptr(self.truncated), _ptr(self.status), int(nthreads))

    def held_encoding(self) -> np.ndarray:
        """(B, W, H, 3) x-major encodings of what each Box cell holds (zeros without held planes)."""
        W, H = self.W, self.H
        if self.hty is None:
            return np.zeros((self.B, W, H, 3), np.uint8)
        return np.stack([p[:, : W * H].reshape(self.B, H, W).transpose(0, 2, 1) for p in (self.hty, self.hco, self.hst)],
                        axis=-1)


class OracleEnv:
    """Single env stepped by the oracle's restatement of MiniGridEnv.step (mutable state)."""

    def __init__(self, enc: np.ndarray, agent, max_steps: int, see_through: bool, view=7, held=None):
        # enc is the reference's x-major (W, H, 3) encode; planes are row-major (H, W).  held: the
        # same layout for what each Box cell holds (Box(contains=...), type 0 = nothing), optional
        enc = np.asarray(enc, np.uint8)
        self.ty = np.ascontiguousarray(enc[:, :, 0].T)
        self.co = np.ascontiguousarray(enc[:, :, 1].T)
        self.st = np.ascontiguousarray(enc[:, :, 2].T)
        self.H, self.W = self.ty.shape
        self.hty = self.hco = self.hst = None
        self.held_carry = np.zeros(3, np.int32)
        if held is not None:
            held = np.asarray(held, np.uint8)
            self.hty, self.hco, self.hst = (np.ascontiguousarray(held[:, :, p].T) for p in range(3))
        self.state = np.array([agent[0], agent[1], agent[2], 0], np.int32)
        self.carry = np.zeros(2, np.int32)
        self.max_steps = int(max_steps)
        self.see_through = bool(see_through)
        self.view = view

    def step(self, action: int):
        img = np.zeros((self.view, self.view, 3), np.uint8)
        r = ctypes.c_double(0)
        te = ctypes.c_int(0)
        tr = ctypes.c_int(0)
        if self.hty is not None:
            rc = lib().orc_step_held(self.W, self.H, _ptr(self.ty), _ptr(self.co), _ptr(self.st), _ptr(self.hty),
                                     _ptr(self.hco), _ptr(self.hst), _ptr(self.held_carry), _ptr(self.state),
                                     _ptr(self.carry), self.max_steps, int(self.see_through), self.view, int(action),
                                     _ptr(img), ctypes.byref(r), ctypes.byref(te), ctypes.byref(tr))
        else:
            rc = lib().orc_step(self.W, self.H, _ptr(self.ty), _ptr(self.co), _ptr(self.st),
                                _ptr(self.state), _ptr(self.carry), self.max_steps,
                                int(self.see_through), self.view, int(action), _ptr(img),
                                ctypes.byref(r), ctypes.byref(te), ctypes.byref(tr))
        if rc == -1:
            raise ValueError(f"Unknown action: {action}")
        if rc != 0:
            raise AssertionError("front cell outside the grid")
        return img, r.value, bool(te.value), bool(tr.value)

    def encode(self) -> np.ndarray:
        return np.stack([self.ty.T, self.co.T, self.st.T], axis=-1)

    def held_encoding(self) -> np.ndarray:
        if self.hty is None:
            return np.zeros((self.W, self.H, 3), np.uint8)
        return np.stack([self.hty.T, self.hco.T, self.hst.T], axis=-1)

    def obs(self):
        return gen_obs((self.ty, self.co, self.st), self.state[:3], self.carry, self.see_through,
                       self.view)
