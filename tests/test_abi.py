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
    assert L.mgdp_abi_version() == _lib.ABI_VERSION == 12
    n = ctypes.c_int32(-1)
    assert L.mgdp_device_count(ctypes.byref(n)) == 0
    assert n.value >= 0
    # argument validation happens before any device work
    assert L.mgdp_vi_create(None, None) == _lib.MGDP_E_INVALID
    assert "null" in _lib.last_error()


def _elf_section(path, name):
    """Bytes of one section of a 64-bit little-endian ELF file."""
    import struct

    b = open(path, "rb").read()
    shoff, = struct.unpack_from("<Q", b, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", b, 0x3A)
    sh = [struct.unpack_from("<IIQQQQIIQQ", b, shoff + i * shentsize) for i in range(shnum)]
    strtab = sh[shstrndx]
    for s in sh:
        nm = b[strtab[4] + s[0]:b.index(b"\0", strtab[4] + s[0])].decode()
        if nm == name:
            return b[s[4]:s[4] + s[5]]
    raise KeyError(name)


def test_code_object_targets_gfx950(tmp_path):
    """Every offload bundle in the library's fatbin carries a gfx950 code object.  The bundles are
    compressed (build.py: --offload-compress), so the target is read back by clang-offload-bundler."""
    import shutil
    import struct
    import subprocess

    fat = _elf_section(_lib.lib_path(), ".hip_fatbin")
    starts, i = [], 0
    while True:
        hits = [x for x in (fat.find(b"CCOB", i), fat.find(b"__CLANG_OFFLOAD_BUNDLE__", i)) if x >= 0]
        if not hits:
            break
        starts.append(min(hits))
        i = min(hits) + 4
    assert len(starts) >= 3  # vi, envs, gen (lib.cpp / comm.cpp carry no device code)
    bundler = shutil.which("clang-offload-bundler") or "/opt/rocm/lib/llvm/bin/clang-offload-bundler"
    for n, s in enumerate(starts):
        if fat[s:s + 4] == b"CCOB":
            ver = struct.unpack_from("<H", fat, s + 4)[0]
            size = struct.unpack_from("<Q" if ver >= 3 else "<I", fat, s + 8)[0]
        else:
            size = (starts[n + 1] if n + 1 < len(starts) else len(fat)) - s
        chunk = tmp_path / f"b{n}.bin"
        chunk.write_bytes(fat[s:s + size])
        if not os.path.exists(bundler):
            if fat[s:s + 4] == b"CCOB":
                pytest.skip("clang-offload-bundler not found: compressed bundles cannot be listed")
            assert b"gfx950" in fat[s:s + size]
            continue
        out = subprocess.run([bundler, "--list", "--type=o", f"--input={chunk}"], capture_output=True, text=True,
                             check=True).stdout
        assert "hipv4-amdgcn-amd-amdhsa--gfx950" in out, out


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
