"""ctypes binding of libmgdp.so (include/mgdp.h) -- the only route from Python to the HIP kernels.

There is no CPU fallback: if the library is missing or no GPU is visible, the product raises.
"""
from __future__ import annotations

import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
# MGDP_LIB: an alternative build of the same sources (tools/ experiments with compile-time knobs)
LIB_PATH = os.environ.get("MGDP_LIB") or os.path.join(HERE, "libmgdp.so")

ABI_VERSION = 12
MGDP_OK = 0
MGDP_E_INVALID = -1
MGDP_E_HIP = -2
MGDP_E_UNSUPPORTED = -3
MGDP_E_ACTION = -4
MGDP_E_BOUNDS = -5

MODEL_XYD = 0
MODEL_DOORKEY = 1
F32 = 0
F64 = 1
METHOD_FUSED = 0
METHOD_SWEEP = 1
MAP_CELL = 0
MAP_SA = 1


class MgdpError(RuntimeError):
    pass


class ViDesc(ctypes.Structure):
    _fields_ = [
        ("model", ctypes.c_int32),
        ("dtype", ctypes.c_int32),
        ("method", ctypes.c_int32),
        ("mapping", ctypes.c_int32),
        ("B", ctypes.c_int32),
        ("W", ctypes.c_int32),
        ("H", ctypes.c_int32),
        ("max_sweeps", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("gamma", ctypes.c_double),
        ("tol", ctypes.c_double),
        ("slip_p", ctypes.c_double),
        ("horizon", ctypes.c_int32),
        ("lava_mode", ctypes.c_int32),
        ("flags", ctypes.c_int32),
        ("reserved2", ctypes.c_int32),
        ("death_cost", ctypes.c_double),
    ]


class GenDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in
                ("family", "W", "H", "num_crossings", "obstacle", "random_start", "strip2_row", "reserved")]


# name -> (restype, argtypes); the full export list of include/mgdp.h
_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64P = ctypes.POINTER(ctypes.c_int64)
_I32P = ctypes.POINTER(ctypes.c_int32)
_DP = ctypes.POINTER(ctypes.c_double)
SIGNATURES = {
    "mgdp_last_error": (ctypes.c_char_p, []),
    "mgdp_abi_version": (ctypes.c_int, []),
    "mgdp_device_count": (ctypes.c_int, [_I32P]),
    "mgdp_pin_host_thread": (ctypes.c_int, [_I32, _I32P]),
    "mgdp_vi_create": (ctypes.c_int, [ctypes.POINTER(ViDesc), ctypes.POINTER(_P)]),
    "mgdp_vi_destroy": (ctypes.c_int, [_P]),
    "mgdp_vi_set_stream": (ctypes.c_int, [_P, _P]),
    "mgdp_vi_load_cells": (ctypes.c_int, [_P, _P]),
    "mgdp_vi_load_cells_device": (ctypes.c_int, [_P, _P]),
    "mgdp_vi_solve": (ctypes.c_int, [_P, _I32P, _DP, _I32P]),
    "mgdp_vi_solve_last": (ctypes.c_int, [_P, _I32P, _DP, _I32P]),
    "mgdp_vi_resume": (ctypes.c_int, [_P, _P, _I32, ctypes.c_double, _I32P, _DP, _I32P]),
    "mgdp_vi_reset": (ctypes.c_int, [_P]),
    "mgdp_vi_run_local": (ctypes.c_int, [_P, _I32P]),
    "mgdp_vi_run_to": (ctypes.c_int, [_P, _I32, _DP]),
    "mgdp_vi_sweep": (ctypes.c_int, [_P, _DP]),
    "mgdp_vi_finish": (ctypes.c_int, [_P, _I32]),
    "mgdp_vi_run_local_dev": (ctypes.c_int, [_P, _P]),
    "mgdp_vi_run_to_dev": (ctypes.c_int, [_P, _P, _P]),
    "mgdp_vi_set_result": (ctypes.c_int, [_P, _I32, ctypes.c_double]),
    "mgdp_comm_available": (ctypes.c_int, []),
    "mgdp_comm_unique_id": (ctypes.c_int, [_P]),
    "mgdp_comm_create": (ctypes.c_int, [_P, _I32, _I32, _I32, ctypes.POINTER(_P)]),
    "mgdp_comm_create_host": (ctypes.c_int, [ctypes.c_char_p, _I32, _I32, _I32, ctypes.POINTER(_P)]),
    "mgdp_comm_destroy": (ctypes.c_int, [_P]),
    "mgdp_comm_allreduce_max": (ctypes.c_int, [_P, _P, _I32]),
    "mgdp_comm_stats": (ctypes.c_int, [_P, _I64P, _I32P, _I32P]),
    "mgdp_comm_host_waits": (ctypes.c_int, [_P, _I64P, _I32P]),
    "mgdp_vi_solve_sharded": (ctypes.c_int, [_P, _P, _I32P, _DP, _I32P]),
    "mgdp_vi_run_to_dev_sync": (ctypes.c_int, [_P, _P, _I32P, _DP, _DP]),
    "mgdp_vi_local_result": (ctypes.c_int, [_P, _I32P, _DP, _I32P]),
    "mgdp_vi_get_values": (ctypes.c_int, [_P, _P]),
    "mgdp_vi_get_policy": (ctypes.c_int, [_P, _P]),
    "mgdp_vi_get_dv_trace": (ctypes.c_int, [_P, _P, _I32]),
    "mgdp_vi_get_grid_sweeps": (ctypes.c_int, [_P, _P]),
    "mgdp_vi_device_buffers": (ctypes.c_int, [_P, ctypes.POINTER(_P), ctypes.POINTER(_P)]),
    "mgdp_vi_num_states": (ctypes.c_int, [ctypes.POINTER(ViDesc), _I64P]),
    "mgdp_vi_synchronize": (ctypes.c_int, [_P]),
    "mgdp_vi_enable_timing": (ctypes.c_int, [_P, _I32]),
    "mgdp_vi_kernel_time": (ctypes.c_int, [_P, _DP, _I64P]),
    "mgdp_vi_serve_clock": (ctypes.c_int, [_P, _DP, _DP, _I64P, _DP, _I64P]),
    "mgdp_vi_persistent": (ctypes.c_int, [_P, _I32P]),
    "mgdp_vi_kernel_name": (ctypes.c_char_p, [_P]),
    "mgdp_vi_variant": (ctypes.c_char_p, [_P]),
    "mgdp_vi_get_policy_t": (ctypes.c_int, [_P, _P]),
    "mgdp_gen_grids": (ctypes.c_int, [ctypes.POINTER(GenDesc), _I32, _P, ctypes.c_int64, _I32, _P, _P, _P]),
    "mgdp_gen_grids_host": (ctypes.c_int, [ctypes.POINTER(GenDesc), _I32, ctypes.c_int64, _I32, _P, _P, _P]),
    "mgdp_envs_create": (ctypes.c_int, [_I32, _I32, _I32, _I32, _I32, ctypes.POINTER(_P)]),
    "mgdp_envs_destroy": (ctypes.c_int, [_P]),
    "mgdp_envs_set_stream": (ctypes.c_int, [_P, _P]),
    "mgdp_envs_set_nodeath": (ctypes.c_int, [_P, ctypes.c_uint32, ctypes.c_double]),
    "mgdp_envs_load": (ctypes.c_int, [_P, _P, _P, _P, _P, _P]),
    "mgdp_envs_observe": (ctypes.c_int, [_P, _P, _P]),
    "mgdp_envs_step": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _P]),
    "mgdp_envs_step_device": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _P]),
    "mgdp_envs_enable_timing": (ctypes.c_int, [_P, _I32]),
    "mgdp_envs_kernel_time": (ctypes.c_int, [_P, _DP, _I64P]),
    "mgdp_envs_get_state": (ctypes.c_int, [_P, _P, _P, _P, _P]),
    "mgdp_envs_set_state": (ctypes.c_int, [_P, _P, _P, _P, _P]),
    "mgdp_envs_set_contents": (ctypes.c_int, [_P, _P, _P]),
    "mgdp_envs_get_contents": (ctypes.c_int, [_P, _P, _P]),
}

_lib = None


def lib_path() -> str:
    return LIB_PATH


_RAW = None
_RAW_GIL = None


def raw_fn(name: str, keep_gil: bool = False):
    """`name` from a second handle on the loaded library with no argtypes: for hot calls whose
    arguments are already ctypes objects, so the call skips ctypes' per-argument conversion.
    keep_gil: through ctypes.PyDLL, which does not release and re-take the GIL around the call --
    for calls of a few microseconds only (a served lone-grid solve: 0.12-0.16 us less per call,
    tools/probe_solve_py.py)."""
    global _RAW, _RAW_GIL
    load()  # the checked load (ABI version, symbols) happens once
    if keep_gil:
        if _RAW_GIL is None:
            _RAW_GIL = ctypes.PyDLL(LIB_PATH)
        fn = getattr(_RAW_GIL, name)
    else:
        if _RAW is None:
            _RAW = ctypes.CDLL(LIB_PATH)
        fn = getattr(_RAW, name)
    fn.restype = ctypes.c_int
    return fn


def load():
    """Load libmgdp.so (raises if it has not been built; see minigrid_dynamicprogramming_amd.build)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MgdpError(
            f"{LIB_PATH} is missing: build the HIP library first "
            "(python -c 'import __graft_entry__ as g; g.build()')")
    # PyTorch-ROCm bundles its own HIP runtime under the same SONAME (libamdhip64.so.7) as the one
    # libmgdp links; whichever is loaded first serves both, and torch's GPU init fails ("No HIP GPUs
    # are available") if ours came first.  MGDP_HIP_RUNTIME picks: "torch" (default when torch is
    # installed: torch is imported first, so a later torch import in the process still works),
    # "system" (libmgdp binds /opt/rocm's runtime; torch must then not be used for the GPU in this
    # process).  hip_runtime() reports which file was loaded (bench.py records it).
    if os.environ.get("MGDP_HIP_RUNTIME", "torch") != "system" and "torch" not in sys.modules:
        import importlib.util

        if importlib.util.find_spec("torch") is not None:
            import torch  # noqa: F401
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.mgdp_abi_version() != ABI_VERSION:
        raise MgdpError("libmgdp ABI version mismatch")
    _lib = L
    return L


def hip_runtime() -> str | None:
    """Path of the HIP runtime (libamdhip64) mapped into this process, or None."""
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64" in line:
                    return line.split()[-1]
    except OSError:
        pass
    return None


def last_error() -> str:
    msg = load().mgdp_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str = ""):
    """Map an MGDP status code to the reference's exception types (include/mgdp.h)."""
    if rc == MGDP_OK:
        return
    msg = last_error() or what
    if rc in (MGDP_E_INVALID, MGDP_E_UNSUPPORTED, MGDP_E_ACTION):
        raise ValueError(msg)
    if rc == MGDP_E_BOUNDS:
        raise AssertionError(msg)
    raise MgdpError(f"{what}: {msg} (rc={rc})")


def device_count() -> int:
    n = ctypes.c_int32(0)
    check(load().mgdp_device_count(ctypes.byref(n)), "mgdp_device_count")
    return n.value


def pin_host_thread(device: int = 0) -> int:
    """Restrict the calling thread to the CPUs of `device`'s NUMA node (mgdp_pin_host_thread): call
    it before creating the handle that thread will solve on.  Returns the CPUs kept (0: unchanged)."""
    n = ctypes.c_int32(0)
    check(load().mgdp_pin_host_thread(int(device), ctypes.byref(n)), "mgdp_pin_host_thread")
    return n.value


def require_gpu():
    if device_count() <= 0:
        raise MgdpError("no HIP device visible: the MI355X engine has no CPU fallback")


def ptr(a) -> ctypes.c_void_p:
    """Pointer of a contiguous numpy array or a torch tensor (host or device); ints pass through."""
    if a is None or isinstance(a, int):
        return a
    if hasattr(a, "data_ptr"):
        return ctypes.c_void_p(a.data_ptr())
    return a.ctypes.data_as(ctypes.c_void_p)
