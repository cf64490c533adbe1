"""Multi-rank convergence protocol (minigrid_dynamicprogramming_amd/distributed.py) on CPU with gloo.

Each rank's shard is driven through the same protocol the GPU ranks run over RCCL; here the shard
is backed by the CPU oracle, so the test checks the protocol's host logic: the sharded result must
equal one global Jacobi loop over the whole batch (same sweep count, same V, same pi)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from minigrid_dynamicprogramming_amd.distributed import shard_range, solve_sharded
from oracle import oracle
from tests.golden_util import cells_from_enc, load


class OracleShard:
    """run_local / run_to / sweep / finish semantics of an mgdp_vi handle, computed by the oracle."""

    def __init__(self, cells, model=0, tol=1e-6, max_sweeps=10000, slip=None, dtype="f64"):
        self.cells, self.model, self.tol, self.max_sweeps, self.slip, self.dtype = cells, model, tol, max_sweeps, slip, dtype
        self.k = 0

    def _run(self, k):
        return oracle.value_iteration(self.model, self.cells, tol=-1.0, max_sweeps=k, slip_p=self.slip, dtype=self.dtype)

    def reset(self):
        self.k = 0

    def run_local(self):
        ks = [oracle.value_iteration(self.model, c, tol=self.tol, max_sweeps=self.max_sweeps, slip_p=self.slip,
                                     dtype=self.dtype)["sweeps"] for c in self.cells]
        return max(ks)

    def run_to(self, k):
        self.k = k
        return self._run(k)["dv"]

    def sweep(self):
        self.k += 1
        return self._run(self.k)["dv"]

    def finish(self, k, dv):
        r = self._run(k)
        self.V, self.pi, self.sweeps = r["V"], r["pi"], k


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cells, slip, out):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(len(cells), rank, world)
    shard = OracleShard(cells[lo:hi], slip=slip)
    res = solve_sharded(shard)
    out[rank] = (res["sweeps"], res["allreduces"], shard.V, shard.pi, lo, hi)
    dist.barrier()
    dist.destroy_process_group()


def run_world(cells, world, slip=None):
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, cells, slip, out), nprocs=world, join=True)
    return dict(out)


def test_shard_range_covers_exactly():
    for n in (1, 7, 64, 65536):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


@pytest.mark.parametrize("slip", [None, 0.9])
def test_two_rank_gloo_matches_global_loop(slip):
    g = load("grids_fourrooms.npz")
    cells = np.stack([cells_from_enc(e) for e in g["enc"][:12]])
    ref = oracle.value_iteration(0, cells, slip_p=slip)
    out = run_world(cells, 2, slip)
    for rank, (k, nred, V, pi, lo, hi) in out.items():
        assert k == ref["sweeps"]
        assert nred == 2  # one all-reduce for K, one for dV: the contraction holds in fp64
        np.testing.assert_array_equal(V, ref["V"][lo:hi])
        np.testing.assert_array_equal(pi, ref["pi"][lo:hi])


class _FakeReducer:
    def __init__(self):
        self.calls = 0

    def max(self, x):
        self.calls += 1
        return x


class _NonMonotoneShard:
    """dV at the locally chosen K is still >= tol (a rounding-level contraction violation)."""
    tol, max_sweeps = 1e-6, 100

    def reset(self):
        self.trace = [1.0, 1e-3, 2e-6, 3e-6, 9e-7]

    def run_local(self):
        return 3

    def run_to(self, k):
        self.k = k
        return self.trace[k - 1]

    def sweep(self):
        self.k += 1
        return self.trace[self.k - 1]

    def finish(self, k, dv):
        self.final = (k, dv)


def test_fallback_loop_finds_global_stopping_sweep():
    s = _NonMonotoneShard()
    res = solve_sharded(s, reducer=_FakeReducer())
    assert res["sweeps"] == 5 and res["converged"] and s.final[0] == 5
