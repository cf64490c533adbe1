"""Tabular value iteration over Minigrid grids on MI355X (front end of csrc/vi.hip).

The reference has no DP code; this module implements the build-defined
value iteration of DESIGN.md "A9", whose transition is the reference MiniGridEnv.step
(minigrid/minigrid_env.py:520-583).  Models:
  "xyd"      s = (y*W + x)*4 + dir, 7 actions (Empty, FourRooms, LavaCrossing, SimpleCrossing)
  "doorkey"  s = (((y*W + x)*4 + dir)*2 + has_key)*2 + door_open, 5 action lanes
             (left, right, forward, pickup, toggle)
Optional slip transitions follow StochasticActionWrapper (minigrid/wrappers.py:775-796).
All arithmetic runs in libmgdp.so on the GPU; results are bit-identical to the CPU oracle.
"""
from __future__ import annotations

import atexit
import ctypes
import hashlib
import weakref
from dataclasses import dataclass

import numpy as np

from . import _lib
from .core import COLOR_TO_IDX, OBJECT_TO_IDX

MODELS = {"xyd": _lib.MODEL_XYD, "doorkey": _lib.MODEL_DOORKEY}
DTYPES = {"f32": _lib.F32, "f64": _lib.F64}
METHODS = {"fused": _lib.METHOD_FUSED, "sweep": _lib.METHOD_SWEEP}
MAPPINGS = {"cell": _lib.MAP_CELL, "sa": _lib.MAP_SA}
DOORKEY_ACTIONS = (0, 1, 2, 3, 5)  # DP action lane -> env action (doorkey.py:25-33)


def n_states(model: str, W: int, H: int) -> int:
    return W * H * (4 if model == "xyd" else 16)


def n_actions(model: str) -> int:
    return 7 if model == "xyd" else 5


def state_index(model: str, W: int, x: int, y: int, d: int, has_key: int = 0, door_open: int = 0) -> int:
    s = (y * W + x) * 4 + d
    if model == "doorkey":
        s = (s * 2 + has_key) * 2 + door_open
    return s


def to_cells(grids) -> tuple[np.ndarray, np.ndarray | None]:
    """Normalise grids to (B, H, W) OBJECT_TO_IDX cell codes (+ the (B, W, H, 3) encodings when known).

    Accepts: env objects with .grid, Grid objects (or lists of either), (B, W, H, 3) encodings in
    the reference's x-major Grid.encode() layout, or cell codes (H, W) / (B, H, W)."""
    if isinstance(grids, np.ndarray):
        a = grids
        if a.ndim == 4:  # (B, W, H, 3) encodings
            enc = np.ascontiguousarray(a, dtype=np.uint8)
            return np.ascontiguousarray(enc[..., 0].transpose(0, 2, 1)), enc
        if a.ndim == 2:  # (H, W) cells
            a = a[None]
        if a.ndim != 3:
            raise ValueError("expected (B, W, H, 3) encodings or (B, H, W) / (H, W) cell codes")
        return np.ascontiguousarray(a, dtype=np.uint8), None
    if hasattr(grids, "grid") or hasattr(grids, "encode"):
        grids = [grids]
    encs = []
    for g in grids:
        grid = g.grid if hasattr(g, "grid") else g
        encs.append(grid.encode())
    enc = np.ascontiguousarray(np.stack(encs), dtype=np.uint8)
    return np.ascontiguousarray(enc[..., 0].transpose(0, 2, 1)), enc


def infer_model(cells: np.ndarray) -> str:
    has_door = (cells == OBJECT_TO_IDX["door"]).any()
    has_key = (cells == OBJECT_TO_IDX["key"]).any()
    return "doorkey" if (has_door or has_key) else "xyd"


def check_doorkey_encoding(enc: np.ndarray):
    """DoorKey model preconditions that need colours/states: one LOCKED door, key of its colour."""
    for b in range(enc.shape[0]):
        t = enc[b, :, :, 0]
        door = np.argwhere(t == OBJECT_TO_IDX["door"])
        key = np.argwhere(t == OBJECT_TO_IDX["key"])
        if len(door) != 1 or len(key) != 1:
            raise ValueError(f"grid {b}: the DoorKey model needs exactly one door and one key")
        dx, dy = door[0]
        kx, ky = key[0]
        if enc[b, dx, dy, 2] != 2:
            raise ValueError(f"grid {b}: the DoorKey model starts from a locked door")
        if enc[b, dx, dy, 1] != enc[b, kx, ky, 1]:
            raise ValueError(f"grid {b}: key colour does not match the door")


@dataclass
class VIResult:
    V: np.ndarray        # (B, S) float32 / float64
    pi: np.ndarray       # (B, S) int8 action lane (-1 = absorbing)
    sweeps: int
    converged: bool
    dv: float            # max |V_k - V_{k-1}| at the last sweep
    model: str
    W: int
    H: int

    def value(self, b: int, x: int, y: int, d: int, has_key: int = 0, door_open: int = 0):
        return self.V[b, state_index(self.model, self.W, x, y, d, has_key, door_open)]

    def action(self, b: int, x: int, y: int, d: int, has_key: int = 0, door_open: int = 0) -> int:
        """Greedy env action (Actions id) at a state."""
        lane = int(self.pi[b, state_index(self.model, self.W, x, y, d, has_key, door_open)])
        if lane < 0:
            return -1
        return DOORKEY_ACTIONS[lane] if self.model == "doorkey" else lane


# Handles still open at interpreter exit are destroyed explicitly: a lone-grid handle may keep a
# persistent solver resident on its stream, and destroy() asks it to leave and drains the stream.
_LIVE: "weakref.WeakSet[ValueIteration]" = weakref.WeakSet()


@atexit.register
def _close_live_handles():
    for vi in list(_LIVE):
        try:
            vi.close()
        except Exception:
            pass


class ValueIteration:
    """A batch of B grids resident on one GPU (an mgdp_vi handle); solve() may be called repeatedly.

    method "fused": one workgroup per grid, V in LDS for the whole solve (default; fastest).
    method "sweep": one launch per Jacobi sweep, V double-buffered in HBM.
    mapping "cell": one thread per cell; "sa": one thread per (state, action) + wave max-reduce.
    """

    def __init__(self, grids, model: str = "auto", gamma: float = 0.99, tol: float = 1e-6,
                 slip_p: float | None = None, max_sweeps: int = 10000, dtype: str = "f32",
                 method: str = "fused", mapping: str = "cell", device: int = 0, stream=None,
                 lava: str = "terminal", death_cost: float = -1.0, horizon: int = 0,
                 keep_policy_t: bool = False):
        """lava="nodeath": NoDeath(no_death_types=("lava",), death_cost) semantics
        (wrappers.py:799-872).  horizon=H > 0: finite-horizon DP over step_count with the exact
        _reward() (minigrid_env.py:235-240), H = the env's max_steps; keep_policy_t keeps pi_t."""
        cells, enc = to_cells(grids)
        if model == "auto":
            model = infer_model(cells)
        if model not in MODELS:
            raise ValueError(f"unknown model {model!r}")
        if model == "doorkey" and enc is not None:
            check_doorkey_encoding(enc)
        self.L = _lib.load()
        _lib.require_gpu()
        B, H, W = cells.shape
        self.model, self.B, self.W, self.H = model, B, W, H
        self.S = n_states(model, W, H)
        self.dtype = dtype
        self.np_dtype = np.float32 if dtype == "f32" else np.float64
        self.tol = float(tol)
        self.max_sweeps = int(max_sweeps)
        d = _lib.ViDesc()
        d.model = MODELS[model]
        d.dtype = DTYPES[dtype]
        d.method = METHODS[method]
        d.mapping = MAPPINGS[mapping]
        d.B, d.W, d.H = B, W, H
        d.max_sweeps = self.max_sweeps
        d.device = device
        d.gamma = float(gamma)
        d.tol = float(tol)
        d.slip_p = -1.0 if slip_p is None else float(slip_p)
        if lava not in ("terminal", "nodeath"):
            raise ValueError(f"lava must be 'terminal' or 'nodeath', got {lava!r}")
        d.lava_mode = 1 if lava == "nodeath" else 0
        d.death_cost = float(death_cost)
        d.horizon = int(horizon)
        d.flags = 1 if keep_policy_t else 0
        self.horizon = int(horizon)
        self.method, self.lava = method, lava
        self.desc = d
        self._solve_args = None
        self._live = None  # the last solve()'s ctypes outputs while they are the current result
        self._sharded_args = None
        self._load_dev_fn = None
        h = ctypes.c_void_p()
        _lib.check(self.L.mgdp_vi_create(ctypes.byref(d), ctypes.byref(h)), "mgdp_vi_create")
        self.h = h
        _LIVE.add(self)
        if stream is not None:
            _lib.check(self.L.mgdp_vi_set_stream(h, ctypes.c_void_p(int(stream))), "mgdp_vi_set_stream")
        self.load(cells)

    @property
    def persistent(self) -> bool:
        """Whether solve() is served by the resident vi_serve_kernel (lone grid, fused, cell)."""
        on = ctypes.c_int32(0)
        _lib.check(self.L.mgdp_vi_persistent(self.h, ctypes.byref(on)), "mgdp_vi_persistent")
        return bool(on.value)

    @property
    def kernel_name(self) -> str:
        """The kernel kernel_time() times on this handle, as rocprofv3 lists it."""
        n = self.L.mgdp_vi_kernel_name(self.h)
        if n is None:
            _lib.check(_lib.MGDP_E_INVALID, "mgdp_vi_kernel_name")
        return n.decode()

    @property
    def variant(self) -> str:
        """Which loop of that kernel runs (mgdp_vi_variant): e.g. serve_ew, wave2, dk_rows, dk_half."""
        n = self.L.mgdp_vi_variant(self.h)
        if n is None:
            _lib.check(_lib.MGDP_E_INVALID, "mgdp_vi_variant")
        return n.decode()

    def load(self, grids):
        """Install new grids of the same shape (mgdp_vi_load_cells); the next solve uses them."""
        cells, enc = to_cells(grids)
        if cells.shape != (self.B, self.H, self.W):
            raise ValueError(f"grids of shape {cells.shape} do not match the handle's {(self.B, self.H, self.W)}")
        if self.model == "doorkey" and enc is not None:
            check_doorkey_encoding(enc)
        cells = np.ascontiguousarray(cells, np.uint8)
        _lib.check(self.L.mgdp_vi_load_cells(self.h, _lib.ptr(cells)), "mgdp_vi_load_cells")
        self._cells_digest = hashlib.sha256(cells.tobytes()).hexdigest()  # checkpoint() / resume()
        self.sweeps = 0
        self.converged = False
        self.dv = float("nan")

    def load_device(self, cells_ptr: int):
        """Install new grids from device memory (mgdp_vi_load_cells_device): B*H*W row-major type
        codes at `cells_ptr` (e.g. a torch uint8 tensor's data_ptr()), complete before the call and
        unchanged until the next solve returns.  A resident lone-grid server takes the grid with
        its next request, so this makes no HIP call; the bytes are not validated here."""
        if self._load_dev_fn is None:
            self._load_dev_fn = _lib.raw_fn("mgdp_vi_load_cells_device")
        rc = self._load_dev_fn(self.h, ctypes.c_void_p(int(cells_ptr)))
        if rc:
            _lib.check(rc, "mgdp_vi_load_cells_device")
        self._cells_digest = None  # not read back: a checkpoint of these grids cannot be verified
        self.sweeps = 0
        self.converged = False
        self.dv = float("nan")

    def close(self):
        if getattr(self, "h", None):
            self.L.mgdp_vi_destroy(self.h)
            self.h = None
            self._solve_args = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- single-device solve
    def solve(self, last: bool = False) -> int:
        """Whole solve (mgdp_vi_solve).  last=True (mgdp_vi_solve_last): a resident lone-grid server
        leaves right after this solve instead of idling out; the next solve relaunches it."""
        if self._solve_args is None:  # reused ctypes arguments: nothing converted or allocated per solve
            self._out = (ctypes.c_int32(0), ctypes.c_double(0), ctypes.c_int32(0))
            self._solve_args = (ctypes.c_void_p(self.h.value if isinstance(self.h, ctypes.c_void_p) else self.h),) + \
                tuple(ctypes.byref(o) for o in self._out)
            # a resident lone-grid server answers in ~10 us: keep the GIL across that call
            quick = self.persistent
            self._solve_fn = _lib.raw_fn("mgdp_vi_solve", keep_gil=quick)
            self._solve_last_fn = _lib.raw_fn("mgdp_vi_solve_last", keep_gil=quick)
        rc = (self._solve_last_fn if last else self._solve_fn)(*self._solve_args)
        if rc:
            _lib.check(rc, "mgdp_vi_solve")
        # the result stays in the ctypes outputs (sweeps / dv / converged read them): a served solve
        # takes a few microseconds, and converting and storing three attributes per call was a
        # measurable part of the host's turnaround between requests
        self._live = self._out
        return self._out[0].value

    # sweeps / dv / converged of the last result: read from solve()'s outputs while they are current
    def _result_attr(self, i, name):
        live = self.__dict__.get("_live")
        if live is not None:
            return (live[0].value, live[1].value, bool(live[2].value))[i]
        return self.__dict__[name]

    def _set_result_attr(self, name, v):
        live = self.__dict__.get("_live")
        if live is not None:  # leaving the live outputs: the other two keep their values
            self.__dict__.update(_sweeps=live[0].value, _dv=live[1].value, _converged=bool(live[2].value))
            self.__dict__["_live"] = None
        self.__dict__[name] = v

    sweeps = property(lambda self: self._result_attr(0, "_sweeps"), lambda self, v: self._set_result_attr("_sweeps", v))
    dv = property(lambda self: self._result_attr(1, "_dv"), lambda self, v: self._set_result_attr("_dv", v))
    converged = property(lambda self: self._result_attr(2, "_converged"),
                         lambda self, v: self._set_result_attr("_converged", v))

    def solve_sharded(self, comm) -> int:
        """One sharded solve with the library's own collectives (mgdp_vi_solve_sharded on a
        distributed.LibComm): every rank of the communicator calls it (or joins host-driven)."""
        if self._sharded_args is None or self._sharded_args[1] != comm.handle:
            self._sh_out = (ctypes.c_int32(0), ctypes.c_double(0), ctypes.c_int32(0))
            self._sharded_args = (self.h, comm.handle) + tuple(ctypes.byref(o) for o in self._sh_out)
        _lib.check(self.L.mgdp_vi_solve_sharded(*self._sharded_args), "mgdp_vi_solve_sharded")
        k, dv, conv = self._sh_out
        self.sweeps, self.dv, self.converged = k.value, dv.value, bool(conv.value)
        return self.sweeps

    @property
    def sharded_capable(self) -> bool:
        """Whether mgdp_vi_solve_sharded runs this handle (fused method, no horizon / lava options)."""
        return self.method == "fused" and self.horizon == 0 and self.lava == "terminal"

    # -- multi-device protocol pieces (see distributed.py)
    def reset(self):
        _lib.check(self.L.mgdp_vi_reset(self.h), "mgdp_vi_reset")

    def run_local(self) -> int:
        k = ctypes.c_int32(0)
        _lib.check(self.L.mgdp_vi_run_local(self.h, ctypes.byref(k)), "mgdp_vi_run_local")
        return k.value

    def local_result(self) -> tuple[int, float]:
        """(max sweeps, max |dV| of each grid's last sweep) of the last launch (mgdp_vi_local_result):
        after run_local, dV of every grid at its own stopping sweep."""
        k = ctypes.c_int32(0)
        dv = ctypes.c_double(0)
        _lib.check(self.L.mgdp_vi_local_result(self.h, ctypes.byref(k), ctypes.byref(dv), None),
                   "mgdp_vi_local_result")
        return k.value, dv.value

    def run_to(self, k: int) -> float:
        dv = ctypes.c_double(0)
        _lib.check(self.L.mgdp_vi_run_to(self.h, int(k), ctypes.byref(dv)), "mgdp_vi_run_to")
        return dv.value

    def sweep(self) -> float:
        dv = ctypes.c_double(0)
        _lib.check(self.L.mgdp_vi_sweep(self.h, ctypes.byref(dv)), "mgdp_vi_sweep")
        return dv.value

    # -- the same protocol with device-resident K / dV (distributed.py over RCCL): enqueue only
    @property
    def protocol_device(self):
        """The torch device whose int64 buffers the *_dev steps read and write (None when this handle
        runs the host protocol only: sweep method, horizon or NoDeath options)."""
        if self.desc.method != _lib.METHOD_FUSED or self.horizon > 0 or self.desc.lava_mode != 0:
            return None
        dev = getattr(self, "_protocol_dev", None)
        if dev is None:
            import torch

            dev = self._protocol_dev = torch.device("cuda", self.desc.device)
        return dev

    def bind_stream(self, stream_ptr: int):
        """Launch on this hipStream_t from now on (no-op when it already does)."""
        if getattr(self, "_bound_stream", None) != int(stream_ptr):
            _lib.check(self.L.mgdp_vi_set_stream(self.h, ctypes.c_void_p(int(stream_ptr))), "mgdp_vi_set_stream")
            self._bound_stream = int(stream_ptr)

    def run_local_dev(self, pub):
        """pub: int64 CUDA tensor (or pointer) of 4 words <- {k max, dV bits, k min, 0}."""
        if getattr(self, "_rld_fn", None) is None:
            self._rld_fn = _lib.raw_fn("mgdp_vi_run_local_dev")
        rc = self._rld_fn(self.h, _lib.ptr(pub))
        if rc:
            _lib.check(rc, "mgdp_vi_run_local_dev")

    def run_to_dev(self, k, pub):
        """Every grid to exactly the sweep held by the int64 device word k; results into pub."""
        _lib.check(self.L.mgdp_vi_run_to_dev(self.h, _lib.ptr(k), _lib.ptr(pub)), "mgdp_vi_run_to_dev")

    def run_to_dev_sync(self, kdv) -> tuple[int, float, float]:
        """Every grid to exactly K = kdv[0] (int64 device words, read on the device), then wait on
        the host-mapped result: (K, this shard's dV at K, kdv[1] as a double)."""
        if getattr(self, "_sync_fn", None) is None:
            self._sync_fn = _lib.raw_fn("mgdp_vi_run_to_dev_sync")
            self._sync_out = (ctypes.c_int32(0), ctypes.c_double(0), ctypes.c_double(0))
        k, dv, rule = self._sync_out
        rc = self._sync_fn(self.h, ctypes.c_void_p(kdv.data_ptr()), ctypes.byref(k), ctypes.byref(dv),
                           ctypes.byref(rule))
        if rc:
            _lib.check(rc, "mgdp_vi_run_to_dev_sync")
        return k.value, dv.value, rule.value

    def set_result(self, k: int, dv: float):
        _lib.check(self.L.mgdp_vi_set_result(self.h, int(k), float(dv)), "mgdp_vi_set_result")

    def finish(self, sweeps: int, dv: float):
        _lib.check(self.L.mgdp_vi_finish(self.h, int(sweeps)), "mgdp_vi_finish")
        self.sweeps, self.dv = int(sweeps), float(dv)
        self.converged = dv < self.tol

    # -- results
    def policy_t(self) -> np.ndarray:
        """Finite horizon with keep_policy_t: (H, B, S) int8, pi_t[t] = the greedy lane at step_count t."""
        out = np.empty((self.horizon, self.B, self.S), np.int8)
        _lib.check(self.L.mgdp_vi_get_policy_t(self.h, _lib.ptr(out)), "mgdp_vi_get_policy_t")
        return out

    def grid_sweeps(self) -> np.ndarray:
        """(B,) int32: the sweeps each grid executed (mgdp_vi_get_grid_sweeps) -- its own stopping
        sweep if it ended at an exact fixed point (complete for the global K), else K."""
        k = np.empty(self.B, np.int32)
        _lib.check(self.L.mgdp_vi_get_grid_sweeps(self.h, _lib.ptr(k)), "mgdp_vi_get_grid_sweeps")
        return k

    def values(self) -> np.ndarray:
        V = np.empty((self.B, self.S), self.np_dtype)
        _lib.check(self.L.mgdp_vi_get_values(self.h, _lib.ptr(V)), "mgdp_vi_get_values")
        return V

    def policy(self) -> np.ndarray:
        pi = np.empty((self.B, self.S), np.int8)
        _lib.check(self.L.mgdp_vi_get_policy(self.h, _lib.ptr(pi)), "mgdp_vi_get_policy")
        return pi

    # -- checkpoint / resume: Jacobi is memoryless given V_k
    def _ckpt_meta(self) -> dict:
        """What a checkpoint is only valid for: the grids (sha256 of the cells, None after
        load_device) and every parameter the Jacobi trajectory depends on."""
        d = self.desc
        return {"model": self.model, "dtype": self.dtype, "B": self.B, "W": self.W, "H": self.H,
                "gamma": float(d.gamma), "tol": float(d.tol), "slip_p": float(d.slip_p),
                "lava_mode": int(d.lava_mode), "death_cost": float(d.death_cost), "horizon": int(d.horizon),
                "cells_sha256": self._cells_digest}

    def checkpoint(self) -> dict:
        """The state of the last solve: {"V" (B, S), "pi" (B, S), "sweeps", "dv", "converged",
        "meta"}.  A solve stopped by max_sweeps before converging continues from it with resume()
        on a handle of the same grids and parameters whose max_sweeps is larger than the
        checkpoint's sweep count (so not on the capped handle itself), bit-identical to the
        uninterrupted solve."""
        return {"V": self.values(), "pi": self.policy(), "sweeps": int(self.sweeps), "dv": float(self.dv),
                "converged": bool(self.converged), "meta": self._ckpt_meta()}

    def resume(self, ckpt: dict, verify_cells: bool = True) -> int:
        """Continue from checkpoint() output (mgdp_vi_resume); returns the sweeps of the whole solve.
        Refused (ValueError): a converged checkpoint (final), V of another shape or dtype, a
        checkpoint of other grids or parameters (its "meta"), and with verify_cells a handle or
        checkpoint whose cells are unknown (loaded with load_device)."""
        meta = ckpt.get("meta")
        if meta is None:
            raise ValueError("checkpoint has no meta (grids and parameters); refusing to resume blind")
        mine = self._ckpt_meta()
        for key, val in mine.items():
            if key == "cells_sha256":
                continue
            if meta.get(key) != val:
                raise ValueError(f"checkpoint {key}={meta.get(key)!r} does not match the handle's {val!r}")
        if verify_cells:
            if mine["cells_sha256"] is None or meta.get("cells_sha256") is None:
                raise ValueError("cells digest unknown (load_device); pass verify_cells=False to resume anyway")
            if meta["cells_sha256"] != mine["cells_sha256"]:
                raise ValueError("checkpoint was taken on other grids (cells sha256 differs)")
        V = np.asarray(ckpt["V"])
        if V.dtype != self.np_dtype:
            raise ValueError(f"checkpoint V is {V.dtype}, the handle computes in {np.dtype(self.np_dtype)}")
        if V.shape != (self.B, self.S):
            raise ValueError(f"checkpoint V of shape {V.shape} does not match the handle's {(self.B, self.S)}")
        V = np.ascontiguousarray(V)
        k, dv, conv = ctypes.c_int32(0), ctypes.c_double(0), ctypes.c_int32(0)
        _lib.check(self.L.mgdp_vi_resume(self.h, _lib.ptr(V), int(ckpt["sweeps"]), float(ckpt["dv"]), ctypes.byref(k),
                                         ctypes.byref(dv), ctypes.byref(conv)), "mgdp_vi_resume")
        self.sweeps, self.dv, self.converged = k.value, dv.value, bool(conv.value)
        return self.sweeps

    @staticmethod
    def save_checkpoint(path, ckpt: dict) -> None:
        """Write a checkpoint as .npz (plain arrays and a JSON string: np.load needs no pickle)."""
        import json

        np.savez(path, V=ckpt["V"], pi=ckpt["pi"], sweeps=np.int64(ckpt["sweeps"]), dv=np.float64(ckpt["dv"]),
                 converged=np.bool_(ckpt["converged"]), meta=np.str_(json.dumps(ckpt.get("meta"))))

    @staticmethod
    def load_checkpoint(path) -> dict:
        import json

        z = np.load(path)  # allow_pickle=False
        return {"V": z["V"], "pi": z["pi"], "sweeps": int(z["sweeps"]), "dv": float(z["dv"]),
                "converged": bool(z["converged"]), "meta": json.loads(str(z["meta"])) if "meta" in z else None}

    def dv_trace(self) -> np.ndarray:
        t = np.zeros(self.sweeps, np.float64)
        _lib.check(self.L.mgdp_vi_get_dv_trace(self.h, _lib.ptr(t), self.sweeps), "mgdp_vi_get_dv_trace")
        return t

    def result(self) -> VIResult:
        return VIResult(self.values(), self.policy(), self.sweeps, self.converged, self.dv, self.model,
                        self.W, self.H)

    def synchronize(self):
        """Complete all work of the handle (a resident lone-grid server leaves, the stream drains)."""
        _lib.check(self.L.mgdp_vi_synchronize(self.h), "mgdp_vi_synchronize")

    def enable_timing(self, on: bool = True):
        _lib.check(self.L.mgdp_vi_enable_timing(self.h, int(on)), "mgdp_vi_enable_timing")

    def serve_clock(self) -> dict:
        """Shader clock of the persistent lone-grid servers that ran since enable_timing(): each
        launch's s_memtime cycles over its s_memrealtime lifetime (mgdp_vi_serve_clock)."""
        mhz, us, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
        sus, ns = ctypes.c_double(), ctypes.c_int64()
        _lib.check(self.L.mgdp_vi_serve_clock(self.h, ctypes.byref(mhz), ctypes.byref(us), ctypes.byref(n),
                                              ctypes.byref(sus), ctypes.byref(ns)), "mgdp_vi_serve_clock")
        return {"sclk_mhz": mhz.value, "server_us": us.value, "launches": n.value, "gpu_solve_us": sus.value,
                "solves": ns.value}

    def kernel_time(self) -> tuple[float, int]:
        ms = ctypes.c_double(0)
        n = ctypes.c_int64(0)
        _lib.check(self.L.mgdp_vi_kernel_time(self.h, ctypes.byref(ms), ctypes.byref(n)), "mgdp_vi_kernel_time")
        return ms.value, n.value

    @property
    def updates_per_sweep(self) -> int:
        return self.B * self.S * n_actions(self.model)


def value_iteration(grids, **kwargs) -> VIResult:
    """Solve value iteration for one grid or a batch (one global stopping rule) on one GPU."""
    vi = ValueIteration(grids, **kwargs)
    try:
        vi.solve()
        return vi.result()
    finally:
        vi.close()
