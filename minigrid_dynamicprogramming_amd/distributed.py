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

Device protocol (RCCL, fused method): K and dV never visit the host between the steps.  The
shard's two launches publish {k max, dV bits, k min, epoch} into an int64 buffer on the GPU, the
all-reduces run on the same stream (ProcessGroupNCCL orders its stream after the current one and
the current one after the collective), run_to reads K on the device, and the host reads K and dV
ONCE per solve.  Non-negative doubles order like their IEEE-754 bit patterns, so a MAX over the
int64 bits is the MAX over the values.  Host protocol (gloo, sweep method, DP options): one
host-synchronous scalar all-reduce per step.
"""
from __future__ import annotations

import struct
import time

import numpy as np


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block partition of n units over `world` ranks."""
    base, rem = divmod(n, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def bits_to_double(b: int) -> float:
    return struct.unpack("<d", struct.pack("<q", int(b)))[0]


def double_to_bits(x: float) -> int:
    return struct.unpack("<q", struct.pack("<d", float(x)))[0]


class Reducer:
    """MAX all-reduces of the stopping rule, built ONCE per process and reused by every solve.

    device: cuda for the nccl (RCCL) backend, cpu for gloo.  `proto` is the protocol buffer of the
    device path (int64[8]: [0..3] run_local's result, [4..7] run_to's).  Counters: `calls`
    (all-reduces issued), `host_reads` (host round trips of the device path), `wall_s` (host time
    inside the protocol's collectives and its one read), and with `timing` the device time of each
    all-reduce (event pairs on the protocol stream, summed by collect())."""

    def __init__(self, group=None, timing: bool = False):
        import torch
        import torch.distributed as dist

        self.torch = torch
        self.dist = dist
        self.group = group
        backend = dist.get_backend(group)
        self.device = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
        self.buf = torch.zeros(1, dtype=torch.float64, device=self.device)
        self.proto = torch.zeros(8, dtype=torch.int64, device=self.device)
        self.stream = torch.cuda.Stream(device=self.device) if self.device.type == "cuda" else None
        self.timing = timing and self.device.type == "cuda"
        self._events = []
        self.reset_counters()

    def reset_counters(self):
        self.calls = 0
        self.host_reads = 0
        self.wall_s = 0.0
        self.device_ms = 0.0
        self._events = []

    def max(self, x: float) -> float:
        """Host round trip: all-reduce one scalar and read it back."""
        t = time.perf_counter()
        self.buf.fill_(float(x))
        self.dist.all_reduce(self.buf, op=self.dist.ReduceOp.MAX, group=self.group)
        self.calls += 1
        self.host_reads += 1
        v = float(self.buf.item())
        self.wall_s += time.perf_counter() - t
        return v

    def max_(self, t):
        """In-place MAX of a tensor (slice of `proto`), ordered on the current stream, no host read."""
        if self.timing:
            a = self.torch.cuda.Event(enable_timing=True)
            b = self.torch.cuda.Event(enable_timing=True)
            a.record()
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        if self.timing:
            b.record()
            self._events.append((a, b))
        self.calls += 1

    def collect(self) -> float:
        """Fold the recorded all-reduce event pairs into device_ms (after a synchronize)."""
        for a, b in self._events:
            self.device_ms += a.elapsed_time(b)
        self._events = []
        return self.device_ms


# kept for callers of the round-1 name
_Reducer = Reducer


class EmptyShard:
    """A rank that holds no grids (more ranks than grids): it joins every collective with k = 0 and
    dV = 0, so the other ranks' protocol is unchanged."""

    def __init__(self, tol=1e-6, max_sweeps=10000):
        self.tol, self.max_sweeps = tol, max_sweeps
        self.sweeps = 0

    def reset(self):
        pass

    def run_local(self):
        return 0

    def run_to(self, k):
        return 0.0

    def sweep(self):
        return 0.0

    def finish(self, k, dv):
        self.sweeps = k

    protocol_device = None  # follows the reducer (solve_sharded): the same collectives as its peers

    def bind_stream(self, stream_ptr):
        pass

    def run_local_dev(self, pub):
        pub[0:4] = 0

    def run_to_dev(self, k, pub):
        pub[0:4] = 0

    def set_result(self, k, dv):
        pass


def _device_protocol(vi, red):
    p = red.proto
    vi.reset()
    vi.run_local_dev(p[0:4])
    red.max_(p[0:1])                      # K = the slowest grid anywhere
    vi.run_to_dev(p[0:1], p[4:8])         # every grid to exactly K (K read on the device)
    red.max_(p[5:6])                      # dV at K over every rank
    t = time.perf_counter()
    h = p.tolist()                        # the solve's one host read
    red.wall_s += time.perf_counter() - t
    red.host_reads += 1
    k, dv = int(h[0]), bits_to_double(h[5])
    vi.set_result(k, dv)
    return k, dv


def solve_sharded(vi, group=None, reducer=None) -> dict:
    """Run the protocol above on this rank's shard `vi` (a dp.ValueIteration, an EmptyShard, or any
    object with reset/run_local/run_to/sweep/finish and tol/max_sweeps; with protocol_device and
    run_local_dev/run_to_dev/set_result it takes the device path when that device matches the
    reducer's).  Returns sweeps, dv, converged and the all-reduces / host reads of this solve.
    Must be called by every rank of the group; build the Reducer once and pass it in."""
    red = reducer or Reducer(group)
    calls0, reads0 = red.calls, red.host_reads
    dev = red.device if isinstance(vi, EmptyShard) else getattr(vi, "protocol_device", None)
    if dev is not None and dev.type == red.device.type:
        if red.stream is not None:
            vi.bind_stream(red.stream.cuda_stream)
            with red.torch.cuda.stream(red.stream):
                k, dv = _device_protocol(vi, red)
        else:
            k, dv = _device_protocol(vi, red)
    else:
        vi.reset()
        k = int(red.max(vi.run_local()))
        dv = red.max(vi.run_to(k))
    while not (dv < vi.tol) and k < vi.max_sweeps:
        dv = red.max(vi.sweep())
        k += 1
    vi.finish(k, dv)
    return {"sweeps": k, "dv": dv, "converged": dv < vi.tol, "allreduces": red.calls - calls0,
            "host_reads": red.host_reads - reads0}


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
