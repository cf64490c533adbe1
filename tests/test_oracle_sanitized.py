"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer: the oracle's own
golden-vector tests and its batched step / VI entry points re-run in a child python that loads the
sanitizer build (oracle/Makefile `asan`) with libasan preloaded.  Any out-of-bounds access, use
after free or undefined behaviour aborts the child (UBSan is fatal: -fno-sanitize-recover)."""
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

ORACLE = os.path.join(ROOT, "oracle")


def _libasan():
    out = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    return out if os.path.isabs(out) and os.path.exists(out) else None


@pytest.mark.skipif(_libasan() is None, reason="gcc's libasan is not installed")
def test_oracle_golden_suite_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", ORACLE, "asan"], check=True)
    env = dict(os.environ)
    env.update({
        "MGDP_ORACLE_LIB": os.path.join(ORACLE, "libmgdp_oracle_asan.so"),
        "LD_PRELOAD": _libasan(),
        # the interpreter itself is not instrumented: leaks at exit are python's, not the oracle's
        "ASAN_OPTIONS": "detect_leaks=0:abort_on_error=1",
        "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1",
    })
    cmd = [sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
           os.path.join(ROOT, "tests", "test_oracle_golden.py"),
           os.path.join(ROOT, "tests", "test_sanitized_oracle_calls.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=1200)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, tail
