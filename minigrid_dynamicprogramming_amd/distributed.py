"""Value iteration over grid batches sharded across GPUs (one process per GPU, torch.distributed).

Grids are independent units: rank r holds the contiguous block [r*B/G, (r+1)*B/G) of the global
batch and never exchanges V.  The only collective is the global stopping rule of DESIGN.md "A9"
(stop after sweep k when max over ALL grids of |V_k - V_{k-1}| < tol), carried as scalar MAX
all-reduces over RCCL/xGMI (backend "nccl" on ROCm) or gloo on CPU:

    k_r   = run_local()            each grid sweeps until its own |dV| < tol (no communication)
    K     = allreduce_max(k_r)     the slowest grid anywhere
    dv    = allreduce_max(run_to(K))   every grid advanced to exactly K sweeps
    while dv >= tol and K < max_sweeps:  dv = allreduce_max(sweep()); K += 1   (rare fallback)

Each grid's Jacobi trajectory V_0, V_1, ... does not depend on the other grids, so after this
protocol every grid holds exactly the V_K / pi_K that one global loop would produce.  The Bellman
operator is a gamma-contraction in the sup norm, so per-grid |dV| is non-increasing and K is the
global stopping sweep; the fallback loop covers rounding-level violations (fp32).
"""
from __future__ import annotations

import numpy as np


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block partition of n units over `world` ranks."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


class _Reducer:
    def __init__(self, group=None):
        import torch
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        backend = dist.get_backend(group)
        self.device = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
        self.buf = torch.zeros(1, dtype=torch.float64, device=self.device)
        self.calls = 0

    def max(self, x: float) -> float:
        self.buf.fill_(float(x))
        self.dist.all_reduce(self.buf, op=self.dist.ReduceOp.MAX, group=self.group)
        self.calls += 1
        return float(self.buf.item())


def solve_sharded(vi, group=None, reducer=None) -> dict:
    """Run the protocol above on this rank's shard `vi` (a dp.ValueIteration or any object with
    reset/run_local/run_to/sweep/finish and tol/max_sweeps).  Returns sweeps, dv, converged and
    the number of all-reduces issued.  Must be called by every rank of the group."""
    red = reducer or _Reducer(group)
    vi.reset()
    k = int(red.max(vi.run_local()))
    dv = red.max(vi.run_to(k))
    while not (dv < vi.tol) and k < vi.max_sweeps:
        dv = red.max(vi.sweep())
        k += 1
    vi.finish(k, dv)
    return {"sweeps": k, "dv": dv, "converged": dv < vi.tol, "allreduces": red.calls}


def gather_results(V: np.ndarray, group=None):
    """Gather per-rank (B_r, S) arrays onto every rank (test/diagnostic helper; not on the hot path)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    n = torch.tensor([V.shape[0]], dtype=torch.int64)
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    m = int(max(s.item() for s in sizes))
    pad = np.zeros((m,) + V.shape[1:], V.dtype)
    pad[: V.shape[0]] = V
    t = torch.from_numpy(pad)
    outs = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(outs, t, group=group)
    return np.concatenate([o.numpy()[: int(s.item())] for o, s in zip(outs, sizes)])
