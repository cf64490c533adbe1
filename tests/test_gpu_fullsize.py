"""BASELINE batched configs at their full sizes, GPU vs the oracle's full-batch solve.

BASELINE.json configs[2..4]: FourRooms x 4096, LavaCrossingS11N5 x 65536 and DoorKey-16x16 x 65536
reset(seed) grids (seeds 0..B-1), generated on the GPU by csrc/gen.hip -- whose output over exactly
these seed ranges is pinned to the reference's own sha256 digests by
tests/test_gpu_gen.py::test_gpu_grids_match_reference_digests.  One global stopping rule over the
whole batch: the oracle (oracle/mgdp_oracle.c orc_vi, OpenMP over
grids x states) runs the literal global Jacobi loop, so its sweep count is the batch's global
stopping sweep; the GPU must stop at exactly that sweep with V and pi bit-identical on every grid.
Each oracle solve is computed once per (config, dtype) and shared by the GPU methods.
"""
import json
import os
import time

import numpy as np
import pytest

import minigrid_dynamicprogramming_amd as mg
from minigrid_dynamicprogramming_amd import gen
from oracle import oracle

pytestmark = pytest.mark.gpu

CONFIGS = {
    "fourrooms4096": ("MiniGrid-FourRooms-v0", 4096, "xyd"),
    "lava65536": ("MiniGrid-LavaCrossingS11N5-v0", 65536, "xyd"),
    "doorkey16x65536": ("MiniGrid-DoorKey-16x16-v0", 65536, "doorkey"),
    # fp64 DoorKey batches above the in-kernel-reduce limit (512) run the has_key-split loop
    # (fused_dk_half), vi_reduce_multi_kernel and the chained launches: bench.py's f64 side line of
    # doorkey65536 is exactly this path (seeds 0..16383 of the same generator)
    "doorkey16x16384": ("MiniGrid-DoorKey-16x16-v0", 16384, "doorkey"),
}
CASES = [("fourrooms4096", "f32"), ("fourrooms4096", "f64"), ("lava65536", "f32"), ("lava65536", "f64"),
         ("doorkey16x65536", "f32"), ("doorkey16x16384", "f64")]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _threads() -> int:
    # the GPU box's CPU share is 16 (OMP_NUM_THREADS there); affinity shows the whole machine
    return max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16")), len(os.sched_getaffinity(0))))


_cache = {}


def _oracle(name, dtype):
    key = (name, dtype)
    if key not in _cache:
        _cache.clear()  # one config's tables at a time (DoorKey x 65536: ~17 GB of oracle tables)
        env_id, B, model = CONFIGS[name]
        cells = gen.generate(env_id, 0, B, enc=False, cells=True, agent=False)["cells"]
        t = time.perf_counter()
        o = oracle.value_iteration(0 if model == "xyd" else 1, cells, dtype=dtype, nthreads=_threads())
        o["oracle_s"] = time.perf_counter() - t
        _cache[key] = (cells, o)
    return _cache[key]


def _record(name, dtype, method, sweeps, oracle_s):
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    p = os.path.join(out, "fullsize_sweeps.json")
    d = json.load(open(p)) if os.path.exists(p) else {}
    d[f"{name}/{dtype}/{method}"] = {"sweeps": sweeps, "oracle_s": round(oracle_s, 2), "threads": _threads()}
    with open(p, "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("name,dtype", CASES)
def test_full_batch_global_rule_bit_exact(name, dtype):
    cells, o = _oracle(name, dtype)
    _, _, model = CONFIGS[name]
    for method in ("fused", "sweep"):
        vi = mg.ValueIteration(cells, model=model, dtype=dtype, method=method)
        k = vi.solve()
        assert vi.converged
        assert k == o["sweeps"], f"{name} {dtype} {method}: GPU stopped at sweep {k}, oracle at {o['sweeps']}"
        V, pi = vi.values(), vi.policy()
        vi.close()
        bad = np.flatnonzero((V != o["V"]).any(axis=1) | (pi != o["pi"]).any(axis=1))
        assert bad.size == 0, f"{name} {dtype} {method}: {bad.size} grids differ (first {bad[:8]})"
        _record(name, dtype, method, k, o["oracle_s"])
