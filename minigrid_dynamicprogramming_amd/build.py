"""Build libmgdp.so in-tree with hipcc for gfx950 (cross-compiles without a GPU)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.environ.get("MGDP_BUILD_OUT") or os.path.join(HERE, "libmgdp.so")
SOURCES = ["lib.cpp", "vi.hip", "envs.hip", "gen.hip", "comm.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("MGDP_ARCH", "gfx950")

# -ffp-contract=off: no FMA contraction, so fp32/fp64 arithmetic matches the CPU oracle bit for bit.
# Device code: -fno-honor-nans (V, Q and rewards are finite by construction), which lets max/min
# select v_max_f32 directly instead of canonicalising both operands first under IEEE mode.
# Device code: -fno-slp-vectorize -- the SLP vectorizer packed the batched loops' independent f32
# multiplies and differences into v_pk_mul_f32 / v_pk_add_f32, which measured 5-23 % slower on
# MI355X than the scalar form (FourRooms x 4096 1.33 -> 1.64e13 updates/s unpacked;
# profiles/r03_slp_gk/).
# --offload-compress: the gfx950 code objects go into the fatbin compressed (5.4 -> ~2 MB; the HIP
# runtime inflates them once at load), so the library every GPU run pushes stays small.
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-Xarch_device", "-fno-honor-nans",
         "-Xarch_device", "-fno-slp-vectorize", f"--offload-arch={ARCH}", "--offload-compress", "-Wall",
         "-Wno-unused-result"]
LIBS = ["-ldl"]


def _extra_flags() -> list:
    # MGDP_EXTRA_FLAGS: compile-time knobs of an A/B build (e.g. -DMGDP_SERVE_TRACE), with MGDP_BUILD_OUT
    return os.environ.get("MGDP_EXTRA_FLAGS", "").split()


def _stamp_path() -> str:
    return OUT + ".flags"


def needs_build() -> bool:
    """Stale if any source or the header is newer than the library, or the library was built with
    other compile flags (recorded beside it in <OUT>.flags)."""
    if not os.path.exists(OUT):
        return True
    try:
        with open(_stamp_path()) as f:
            if f.read() != " ".join(FLAGS + _extra_flags()):
                return True
    except OSError:
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [
        os.path.join(HERE, "..", "include", "mgdp.h")]
    return any(os.path.getmtime(p) > t for p in deps if os.path.exists(p))


def build(force: bool = False, verbose: bool = False) -> str:
    """Each translation unit is compiled on its own (in parallel: vi.hip alone takes most of the
    time), then linked; every object carries its own gfx950 code object (no relocatable device code)."""
    from concurrent.futures import ThreadPoolExecutor

    if not force and not needs_build():
        return OUT
    import hashlib
    import tempfile

    extra = _extra_flags()
    # objects of one output and flag set never meet another build's: a private directory per build
    # (parallel builds of A/B variants in one folder cannot overwrite each other's .o files)
    tag = hashlib.sha256((OUT + "\0" + " ".join(extra)).encode()).hexdigest()[:12]
    os.makedirs(os.path.join(HERE, "build"), exist_ok=True)
    objdir = tempfile.mkdtemp(prefix=f"obj_{tag}_", dir=os.path.join(HERE, "build"))
    cflags = [f for f in FLAGS if f != "-shared"] + extra
    jobs = []
    for src in SOURCES:
        obj = os.path.join(objdir, os.path.splitext(src)[0] + ".o")
        jobs.append((obj, [HIPCC, *cflags, "-c", "-o", obj, os.path.join(CSRC, src)]))

    def run(cmd):
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)

    with ThreadPoolExecutor(max_workers=min(len(jobs), os.cpu_count() or 1)) as ex:
        list(ex.map(run, [c for _, c in jobs]))
    tmp = f"{OUT}.tmp{os.getpid()}"
    run([HIPCC, *FLAGS, "-o", tmp, *[o for o, _ in jobs], *LIBS])
    os.replace(tmp, OUT)
    with open(_stamp_path(), "w") as f:
        f.write(" ".join(FLAGS + extra))
    import shutil

    shutil.rmtree(objdir, ignore_errors=True)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
