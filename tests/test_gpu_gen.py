"""GPU batched reset(seed) grid generation (csrc/gen.hip) vs the host generators and the
reference's own grid digests.

The host generators are pinned to the reference (tests/test_host_envs.py); the digests were
computed by the reference itself over the BASELINE batch sizes (tests/golden/make_golden*.py).
"""
import hashlib
import json
import os

import numpy as np
import pytest

import minigrid_dynamicprogramming_amd as mg
from minigrid_dynamicprogramming_amd import gen
from tests.golden_util import GOLDEN, digests

pytestmark = pytest.mark.gpu

IDS = sorted(i for i in mg.registry if gen.supported(mg.make(i)))


def test_every_target_family_is_generated():
    fams = {type(mg.make(i)).__name__ for i in IDS}
    assert fams == {"EmptyEnv", "FourRoomsEnv", "CrossingEnv", "DoorKeyEnv", "LavaGapEnv", "DistShiftEnv"}


@pytest.mark.parametrize("env_id", IDS)
def test_gpu_grids_equal_host_generator(env_id):
    env = mg.make(env_id)
    for seed0, B in ((0, 128), (2**31 - 5, 4), (2**32 + 7, 3), (2**40 + 1, 2)):
        out = gen.generate(env_id, seed0, B, cells=True)
        for b in range(B):
            enc, agent = env.generate(seed=seed0 + b)
            np.testing.assert_array_equal(out["enc"][b], enc, err_msg=f"{env_id} seed {seed0 + b}")
            assert tuple(out["agent"][b]) == tuple(agent), (env_id, seed0 + b)
            np.testing.assert_array_equal(out["cells"][b], enc[:, :, 0].T)


def _digest(out):
    h = hashlib.sha256()
    for b in range(out["enc"].shape[0]):
        h.update(out["enc"][b].tobytes() + out["agent"][b].astype(np.int32).tobytes())
    return h.hexdigest()


@pytest.mark.parametrize("name,env_id", [("fourrooms", "MiniGrid-FourRooms-v0"),
                                         ("lava11n5", "MiniGrid-LavaCrossingS11N5-v0"),
                                         ("doorkey16", "MiniGrid-DoorKey-16x16-v0")])
def test_gpu_grids_match_reference_digests(name, env_id):
    d = digests()[name]
    assert _digest(gen.generate(env_id, 0, d["seeds"])) == d["sha256"]


def test_gpu_lavagap_matches_reference_digest():
    with open(os.path.join(GOLDEN, "digests_f3.json")) as f:
        d = json.load(f)["lavagap7"]
    assert _digest(gen.generate("MiniGrid-LavaGapS7-v0", 0, d["seeds"])) == d["sha256"]


_PIPELINE = r"""
import sys
import torch  # first: PyTorch-ROCm and libmgdp share libamdhip64.so.7, the first one loaded serves both
import numpy as np
sys.path.insert(0, sys.argv[1])
import minigrid_dynamicprogramming_amd as mg
from minigrid_dynamicprogramming_amd import gen, _lib
B, env_id = 4096, "MiniGrid-FourRooms-v0"
env = mg.make(env_id)
cells = torch.empty((B, env.height, env.width), dtype=torch.uint8, device="cuda")
gen.generate_device(env_id, 0, B, cells_ptr=cells, stream=torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
host = gen.generate(env_id, 0, B, enc=False, cells=True, agent=False)["cells"]
assert np.array_equal(cells.cpu().numpy(), host)
vi = mg.ValueIteration(host, dtype="f32")
k_host = vi.solve()
V_host = vi.values()
_lib.check(vi.L.mgdp_vi_load_cells_device(vi.h, _lib.ptr(cells)), "mgdp_vi_load_cells_device")
assert vi.solve() == k_host
assert np.array_equal(vi.values(), V_host)
vi.close()
print("pipeline ok")
"""


def test_device_pipeline_generate_then_solve():
    """Grids generated into device memory (a torch CUDA tensor) feed the solver without a host
    round trip (own process: torch must be imported before libmgdp is first loaded)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _PIPELINE, root], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "pipeline ok" in r.stdout, r.stdout + r.stderr
