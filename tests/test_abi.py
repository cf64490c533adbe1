"""The C-ABI boundary: libmgdp.so builds for gfx950, loads, and exports every symbol of include/mgdp.h.

CPU-only: no compute calls (there is no GPU in the build container)."""
import ctypes
import os
import re

import pytest

from minigrid_dynamicprogramming_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "mgdp.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mgdp_\w+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    L = _lib.load()
    names = header_functions()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert set(names) == set(_lib.SIGNATURES), set(names) ^ set(_lib.SIGNATURES)


def test_abi_version_and_error_string():
    L = _lib.load()
    assert L.mgdp_abi_version() == _lib.ABI_VERSION == 11
    n = ctypes.c_int32(-1)
    assert L.mgdp_device_count(ctypes.byref(n)) == 0
    assert n.value >= 0
    # argument validation happens before any device work
    assert L.mgdp_vi_create(None, None) == _lib.MGDP_E_INVALID
    assert "null" in _lib.last_error()


def test_code_object_targets_gfx950():
    data = open(_lib.lib_path(), "rb").read()
    assert b"gfx950" in data


def test_desc_struct_layout_matches_header():
    # int32 x 10, 3 doubles, int32 x 4, 1 double
    assert ctypes.sizeof(_lib.ViDesc) == 10 * 4 + 3 * 8 + 4 * 4 + 8
    assert _lib.ViDesc.gamma.offset == 40
    assert _lib.ViDesc.horizon.offset == 64 and _lib.ViDesc.death_cost.offset == 80


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="GPU present: the no-GPU error path is not reachable")
def test_pin_host_thread_rejects_missing_device():
    n = ctypes.c_int32(-1)
    assert _lib.load().mgdp_pin_host_thread(0, ctypes.byref(n)) == _lib.MGDP_E_INVALID
    assert n.value == 0
    assert _lib.load().mgdp_pin_host_thread(0, None) == _lib.MGDP_E_INVALID


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="GPU present: the no-GPU error path is not reachable")
def test_product_fails_loudly_without_gpu():
    import numpy as np

    import minigrid_dynamicprogramming_amd as mg

    with pytest.raises(_lib.MgdpError):
        mg.ValueIteration(np.full((1, 5, 5), 2, np.uint8))
