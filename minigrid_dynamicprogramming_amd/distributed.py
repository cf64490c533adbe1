"""Value iteration over grid batches sharded across GPUs (one process per GPU, torch.distributed).

Grids are independent units: rank r holds the contiguous block [r*B/G, (r+1)*B/G) of the global
batch and never exchanges V.  The only collective is the global stopping rule of DESIGN.md "A9"
(stop after sweep k when max over ALL grids of |V_k - V_{k-1}| < tol), carried as MAX all-reduces
of two scalars over RCCL/xGMI (backend "nccl" on ROCm) or gloo on CPU:

    k_r, e_r = run_local()             each grid sweeps until its own |dV| < tol (no communication);
                                       e_r = max |dV| of the shard's grids at their own last sweeps
    K, E  = allreduce_max(k_r, e_r)    the slowest grid anywhere, and the largest own-rule dV
    dv_r  = run_to(K)                  every grid advanced to exactly K sweeps
    dv    = 0 if E == 0 else allreduce_max(dv_r)
    while dv >= tol and K < max_sweeps:  dv = allreduce_max(sweep()); K += 1   (rare fallback)

Each grid's Jacobi trajectory V_0, V_1, ... does not depend on the other grids, so after this
protocol every grid holds exactly the V_K / pi_K that one global loop would produce.  The Bellman
operator is a gamma-contraction in the sup norm, so per-grid |dV| is non-increasing and K is the
global stopping sweep; the fallback loop covers rounding-level violations (fp32).  E == 0 means
every grid stopped its own rule at an exact fixed point (V_k equal to V_{k-1} bit for bit; a sweep
is a function of V alone), so every later sweep reproduces it and dV at K is 0 on every rank: the
second all-reduce is skipped, and a deterministic batch (the shortest-path values settle exactly)
needs ONE collective per solve.

Device protocol (RCCL, fused method): K and E never visit the host before run_to.  The shard's
run_local launch publishes {k max, dV bits, k min, 0} into an int64 buffer on the GPU, the
all-reduce of its first two words runs on the same stream (ProcessGroupNCCL orders its stream after
the current one and the current one after the collective), run_to reads K on the device and its
result comes back through host-mapped memory with E (mgdp_vi_run_to_dev_sync): one host wait per
solve and no stream synchronisation.  Non-negative doubles order like their IEEE-754 bit patterns,
so a MAX over the int64 bits is the MAX over the values.  Host protocol (gloo, sweep method, DP
options, empty shards): the same collectives on the same int64 words, driven from the host, so each
rank picks its path from its own shard alone and no agreement collective is needed.
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
    device path (int64[8]: [0..3] run_local's result, [5] run_to's dV when it is all-reduced).  Counters: `calls`
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
        self.buf2 = torch.zeros(2, dtype=torch.float64, device=self.device)
        self.proto = torch.zeros(8, dtype=torch.int64, device=self.device)
        # the protocol's views of it, made once (a slice is a new tensor object on every use)
        self.p_local, self.p_kd, self.p_dv = self.proto[0:4], self.proto[0:2], self.proto[5:6]
        # the group's allreduce with prebuilt options: dist.all_reduce's argument checks cost more host
        # time per call than issuing the collective (same collective, same stream ordering: wait())
        self._pg = group if group is not None else dist.group.WORLD
        self._opts_max = dist.AllreduceOptions()
        self._opts_max.reduceOp = dist.ReduceOp.MAX
        if hasattr(self._opts_max, "asyncOp"):  # synchronous: RCCL runs on the current stream itself
            self._opts_max.asyncOp = False
        self.stream = torch.cuda.Stream(device=self.device) if self.device.type == "cuda" else None
        # entering / leaving the protocol stream per solve: torch's StreamContext costs ~6 us of
        # Python per solve; its two C calls directly (the context manager when they are absent)
        self._get_stream = getattr(torch._C, "_cuda_getCurrentStream", None)
        self._set_stream = getattr(torch._C, "_cuda_setStream", None)
        if self.stream is not None:
            self.stream_ptr = int(self.stream.cuda_stream)
            self._stream_ids = (self.stream.stream_id, self.stream.device_index, self.stream.device_type)
        self.timing = timing and self.device.type == "cuda"
        self._events = []
        self.reset_counters()

    def enter_stream(self):
        """Make the protocol stream current; returns what exit_stream needs to restore the caller's."""
        if self._get_stream is None or self._set_stream is None:
            ctx = self.torch.cuda.stream(self.stream)
            ctx.__enter__()
            return ctx
        prev = self._get_stream(self.device.index)
        self._set_stream(*self._stream_ids)
        return prev

    def exit_stream(self, prev):
        if isinstance(prev, tuple):
            self._set_stream(*prev)
        else:
            prev.__exit__(None, None, None)

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
        self._all_reduce_max(self.buf)
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
        self._all_reduce_max(t)
        if self.timing:
            b.record()
            self._events.append((a, b))
        self.calls += 1

    def _all_reduce_max(self, t):
        work = self._pg.allreduce([t], self._opts_max)
        if work is not None:
            work.wait()

    def collect(self) -> float:
        """Fold the recorded all-reduce event pairs into device_ms (after a synchronize)."""
        for a, b in self._events:
            self.device_ms += a.elapsed_time(b)
        self._events = []
        return self.device_ms


# kept for callers of the round-1 name
_Reducer = Reducer


class LibComm:
    """The library's own communicator (mgdp_comm_*, include/mgdp.h ABI 11): RCCL over xGMI called
    from libmgdp, so a sharded solve is ONE C call per rank (mgdp_vi_solve_sharded) with its
    collectives enqueued on the handle's stream -- no torch.distributed call, stream switch or
    Python between the launches.  Bootstrapped once per process over a torch.distributed group
    (gloo or nccl): rank 0's 128-byte ncclUniqueId is broadcast to every rank.  Ranks whose shard
    cannot run the device protocol (empty shards, the sweep method, DP options) join the same
    collectives host-driven (mgdp_comm_allreduce_max); see solve_sharded.

    kind="host": the host communicator (mgdp_comm_create_host, ABI 12) -- the same C calls, their
    collectives through a shared-memory segment, for ranks that share one GPU (RCCL refuses them):
    the multi-rank tests of mgdp_vi_solve_sharded.  The constructor is collective; call
    LibComm.available() on every rank and agree first (bench.py does)."""

    @staticmethod
    def available() -> bool:
        """Whether librccl loads in this process (mgdp_comm_available): a local check, no communication."""
        from . import _lib

        return _lib.load().mgdp_comm_available() == 0

    def __init__(self, group=None, device: int | None = None, kind: str = "rccl"):
        import ctypes
        import os
        import uuid

        import torch
        import torch.distributed as dist

        from . import _lib

        self._lib, self._ct = _lib, ctypes
        L = _lib.load()
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self.device = torch.cuda.current_device() if device is None else int(device)
        self.kind = kind
        src = 0 if group is None else dist.get_global_rank(group, 0)
        h = ctypes.c_void_p()
        if kind == "host":
            # a fresh segment name from rank 0; every rank opens it, then it is unlinked (the mappings stay)
            obj = [f"/mgdp_comm_{os.getpid()}_{uuid.uuid4().hex[:12]}" if self.rank == 0 else None]
            dist.broadcast_object_list(obj, src=src, group=group)
            _lib.check(L.mgdp_comm_create_host(obj[0].encode(), self.world, self.rank, self.device, ctypes.byref(h)),
                       "mgdp_comm_create_host")
            dist.barrier(group=group)
            if self.rank == 0:
                try:
                    os.remove("/dev/shm" + obj[0])
                except OSError:
                    pass
        elif kind == "rccl":
            uid = (ctypes.c_uint8 * 128)()
            if self.rank == 0:
                _lib.check(L.mgdp_comm_unique_id(uid), "mgdp_comm_unique_id")
            obj = [bytes(uid) if self.rank == 0 else None]
            dist.broadcast_object_list(obj, src=src, group=group)
            uid = (ctypes.c_uint8 * 128).from_buffer_copy(obj[0])
            _lib.check(L.mgdp_comm_create(uid, self.world, self.rank, self.device, ctypes.byref(h)), "mgdp_comm_create")
        else:
            raise ValueError(f"kind must be 'rccl' or 'host', not {kind!r}")
        self.handle = h
        self._words = (ctypes.c_int64 * 8)()
        # Reducer-like counters for bench.py's collectives block (no per-collective events: the
        # collectives run inside the C call)
        self.device = torch.device("cuda", self.device)
        self.timing = False
        self.reset_counters()

    def reset_counters(self):
        live = getattr(self, "handle", None) is not None
        self._base = self.allreduces if live else 0
        self._wbase = self.host_waits if live else 0
        self.wall_s = 0.0
        self.device_ms = 0.0

    @property
    def calls(self) -> int:
        return self.allreduces - self._base

    @property
    def host_reads(self) -> int:
        """Host waits on the GPU since reset_counters (mgdp_comm_host_waits): the library counts them."""
        return self.host_waits - self._wbase

    @property
    def host_waits(self) -> int:
        c = self._ct.c_int64(0)
        self._lib.check(self._lib.load().mgdp_comm_host_waits(self.handle, self._ct.byref(c), None),
                        "mgdp_comm_host_waits")
        return int(c.value)

    def collect(self) -> float:
        return self.device_ms

    def allreduce_max(self, vals) -> list:
        """Synchronous MAX all-reduce of up to 8 int64 host values (mgdp_comm_allreduce_max)."""
        n = len(vals)
        for i, v in enumerate(vals):
            self._words[i] = int(v)
        self._lib.check(self._lib.load().mgdp_comm_allreduce_max(self.handle, self._words, n), "mgdp_comm_allreduce_max")
        return [int(self._words[i]) for i in range(n)]

    @property
    def allreduces(self) -> int:
        c = self._ct.c_int64(0)
        self._lib.check(self._lib.load().mgdp_comm_stats(self.handle, self._ct.byref(c), None, None), "mgdp_comm_stats")
        return int(c.value)

    def close(self):
        if getattr(self, "handle", None) is not None:
            self._lib.load().mgdp_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 -- interpreter teardown
            pass


def _lib_host_protocol(vi, comm):
    """The collectives of mgdp_vi_solve_sharded driven from the host, for a rank whose shard cannot
    run it (EmptyShard, sweep method, DP options): {k_r, own-rule dV bits} (2 words), then dV(K)
    (1 word) only if the all-reduced dV bits are non-zero -- same words, same order as the C side."""
    vi.reset()
    k_loc, e_loc = _local(vi)
    K, e_bits = comm.allreduce_max([int(k_loc), double_to_bits(e_loc)])
    k = int(K)
    dv = vi.run_to(k)
    if bits_to_double(e_bits) == 0.0:
        if dv != 0.0:
            raise RuntimeError(f"fixed-point invariant violated: dV at sweep {k} is {dv!r}")
    else:
        dv = bits_to_double(comm.allreduce_max([double_to_bits(dv)])[0])
    return k, dv


class EmptyShard:
    """A rank that holds no grids (more ranks than grids): it joins every collective with k = 0 and
    dV = 0, so the other ranks' protocol is unchanged; it takes whichever protocol its peers take."""

    def __init__(self, tol=1e-6, max_sweeps=10000):
        self.tol, self.max_sweeps = tol, max_sweeps
        self.sweeps = 0

    def reset(self):
        pass

    def run_local(self):
        return 0

    def local_result(self):
        return 0, 0.0

    def run_to(self, k):
        return 0.0

    def sweep(self):
        return 0.0

    def finish(self, k, dv):
        self.sweeps = k

    protocol_device = None  # the host path's collectives (the same as the device path's)

    def bind_stream(self, stream_ptr):
        pass

    def run_local_dev(self, pub):
        pub[0:4] = 0

    def run_to_dev_sync(self, kdv):
        h = kdv.tolist()
        return int(h[0]), 0.0, bits_to_double(h[1])

    def set_result(self, k, dv):
        pass


def _device_capable(vi, red) -> bool:
    """Whether THIS rank's shard can run the device protocol on this reducer (its protocol device is
    the reducer's: GPU handles under RCCL).  A per-rank choice with no agreement collective: both
    protocols issue the same collectives (int64 words of `red.proto`, see solve_sharded), so peers
    may differ (an EmptyShard, a sweep-method or DP-option handle next to fused handles)."""
    if isinstance(vi, EmptyShard):
        return False
    dev = getattr(vi, "protocol_device", None)
    return dev is not None and dev.type == red.device.type


def _device_protocol(vi, red):
    p = red.proto
    vi.reset()
    vi.run_local_dev(red.p_local)         # {k max, own-rule dV bits, k min, 0}
    red.max_(red.p_kd)                    # K = the slowest grid anywhere, E = the largest own-rule dV
    t = time.perf_counter()
    k, dv, rule = vi.run_to_dev_sync(red.p_kd)  # the gate (or run_to K); the solve's one host wait
    red.wall_s += time.perf_counter() - t
    red.host_reads += 1
    if rule == 0.0:                       # every grid everywhere at an exact fixed point: dV(K) = 0
        if dv != 0.0:
            raise RuntimeError(f"fixed-point invariant violated: dV at sweep {k} is {dv!r} after an exact "
                               "fixed point on every rank")
    else:
        red.p_dv.fill_(double_to_bits(dv))
        red.max_(red.p_dv)                # dV at K over every rank
        t = time.perf_counter()
        dv = bits_to_double(int(p[5].item()))
        red.wall_s += time.perf_counter() - t
        red.host_reads += 1
    vi.set_result(k, dv)
    return k, dv


def _host_protocol(vi, red):
    """The device protocol's collectives, driven from the host: {k_r, own-rule dV bits} into
    red.proto[0:2], MAX all-reduce, read back; run_to(K); dV at K through red.proto[5] unless every
    grid everywhere stopped at an exact fixed point.  Same tensors, dtypes and order as
    _device_protocol, so ranks on either path meet in the same collectives."""
    p = red.proto
    vi.reset()
    k_loc, e_loc = _local(vi)
    p[0:2].copy_(red.torch.tensor([int(k_loc), double_to_bits(e_loc)], dtype=red.torch.int64))
    red.max_(red.p_kd)
    t = time.perf_counter()
    K, e_bits = red.p_kd.tolist()
    red.wall_s += time.perf_counter() - t
    red.host_reads += 1
    k = int(K)
    dv = vi.run_to(k)
    if bits_to_double(e_bits) == 0.0:
        if dv != 0.0:
            raise RuntimeError(f"fixed-point invariant violated: dV at sweep {k} is {dv!r}")
    else:
        red.p_dv.fill_(double_to_bits(dv))
        red.max_(red.p_dv)
        t = time.perf_counter()
        dv = bits_to_double(int(p[5].item()))
        red.wall_s += time.perf_counter() - t
        red.host_reads += 1
    return k, dv


def _local(vi):
    """(k_local, own-rule dV) after run_local; a shard without local_result reports dV as unknown."""
    k = vi.run_local()
    lr = getattr(vi, "local_result", None)
    return (k, float("inf")) if lr is None else (k, float(lr()[1]))


def solve_sharded(vi, group=None, reducer=None, comm=None) -> dict:
    """Run the protocol above on this rank's shard `vi` (a dp.ValueIteration, an EmptyShard, or any
    object with reset/run_local/run_to/sweep/finish and tol/max_sweeps, optionally local_result;
    with protocol_device and run_local_dev/run_to_dev_sync/set_result it can take the device path).
    Returns sweeps, dv, converged and the all-reduces / host reads of this solve (the one-time
    protocol agreement not counted).  Must be called by every rank of the group; build the Reducer
    once and pass it in.  comm (a LibComm, built once, passed by EVERY rank or by none): the
    library's own collectives -- one mgdp_vi_solve_sharded call per solve on ranks whose shard can
    run it, the same collectives host-driven on the others."""
    if comm is not None:
        n0, w0 = comm.allreduces, comm.host_waits
        if getattr(vi, "sharded_capable", False):
            k = vi.solve_sharded(comm)
            return {"sweeps": k, "dv": vi.dv, "converged": vi.converged, "allreduces": comm.allreduces - n0,
                    "host_reads": comm.host_waits - w0, "protocol": "lib"}
        k, dv = _lib_host_protocol(vi, comm)
        while not (dv < vi.tol) and k < vi.max_sweeps:
            dv = bits_to_double(comm.allreduce_max([double_to_bits(vi.sweep())])[0])
            k += 1
        vi.finish(k, dv)
        return {"sweeps": k, "dv": dv, "converged": dv < vi.tol, "allreduces": comm.allreduces - n0,
                "host_reads": comm.host_waits - w0, "protocol": "lib-host"}
    red = reducer or Reducer(group)
    device = _device_capable(vi, red)
    calls0, reads0 = red.calls, red.host_reads
    if device:
        if red.stream is not None:
            vi.bind_stream(red.stream_ptr)
            prev = red.enter_stream()
            try:
                k, dv = _device_protocol(vi, red)
            finally:
                red.exit_stream(prev)
        else:
            k, dv = _device_protocol(vi, red)
    else:
        k, dv = _host_protocol(vi, red)
    while not (dv < vi.tol) and k < vi.max_sweeps:
        dv = red.max(vi.sweep())
        k += 1
    vi.finish(k, dv)
    return {"sweeps": k, "dv": dv, "converged": dv < vi.tol, "allreduces": red.calls - calls0,
            "host_reads": red.host_reads - reads0, "protocol": "device" if device else "host"}


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
