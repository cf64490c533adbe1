import os
import sys

import pytest

try:  # before libmgdp: PyTorch-ROCm's bundled HIP runtime must be the one loaded (see _lib.load)
    import torch  # noqa: F401
except ImportError:
    pass

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def has_gpu() -> bool:
    return os.path.exists("/dev/kfd")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
