"""Multi-rank convergence protocol (minigrid_dynamicprogramming_amd/distributed.py) on CPU with gloo.

Each rank's shard is driven through the same protocol the GPU ranks run over RCCL; here the shard
is backed by the CPU oracle, so the test checks the protocol's host logic: the sharded result must
equal one global Jacobi loop over the whole batch (same sweep count, same V, same pi)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from minigrid_dynamicprogramming_amd.distributed import (EmptyShard, Reducer, bits_to_double, double_to_bits,
                                                         shard_range, solve_sharded)
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
        rs = [oracle.value_iteration(self.model, c, tol=self.tol, max_sweeps=self.max_sweeps, slip_p=self.slip,
                                     dtype=self.dtype) for c in self.cells]
        self._local = (max(r["sweeps"] for r in rs), max(r["dv"] for r in rs))
        return self._local[0]

    def local_result(self):
        return self._local

    def run_to(self, k):
        self.k = k
        return self._run(k)["dv"]

    def sweep(self):
        self.k += 1
        return self._run(self.k)["dv"]

    def finish(self, k, dv):
        r = self._run(k)
        self.V, self.pi, self.sweeps = r["V"], r["pi"], k


class DevOracleShard(OracleShard):
    """The device-protocol steps of the shard (run_local_dev / run_to_dev / set_result) on CPU int64
    tensors: the words a GPU launch would publish, all-reduced by gloo in place."""

    @property
    def protocol_device(self):
        import torch

        return torch.device("cpu")

    def run_local_dev(self, pub):
        pub[0] = self.run_local()
        pub[1] = double_to_bits(self._local[1])
        pub[2] = 0
        pub[3] = 1

    def run_to_dev_sync(self, kdv):
        kk = int(kdv[0])
        return kk, self.run_to(kk), bits_to_double(int(kdv[1]))

    def set_result(self, k, dv):
        self.k = k


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cells, slip, out, device_proto=False, solves=1):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(len(cells), rank, world)
    red = Reducer()  # built once, reused by every solve
    if hi == lo:
        shard = EmptyShard()
    else:
        # device_proto "mixed": odd ranks' shards can only take the host protocol
        dev = device_proto is True or (device_proto == "mixed" and rank % 2 == 0)
        shard = (DevOracleShard if dev else OracleShard)(cells[lo:hi], slip=slip)
    for _ in range(solves):
        res = solve_sharded(shard, reducer=red)
    V = getattr(shard, "V", None)
    pi = getattr(shard, "pi", None)
    out[rank] = (res["sweeps"], res["allreduces"], V, pi, lo, hi, res["host_reads"], red.calls,
                 res["protocol"] == "device")
    dist.barrier()
    dist.destroy_process_group()


def run_world(cells, world, slip=None, device_proto=False, solves=1):
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, cells, slip, out, device_proto, solves), nprocs=world, join=True)
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
    for rank, (k, nred, V, pi, lo, hi, reads, _, proto) in out.items():
        assert k == ref["sweeps"]
        assert proto is False  # gloo + host-only shards: the host protocol on every rank
        # deterministic: every grid ends its own rule at an exact fixed point, so one all-reduce of
        # {K, own-rule dV} settles the solve; slip: a second one for dV at K (the contraction holds in fp64)
        assert nred == (1 if slip is None else 2)
        assert reads == nred  # host protocol: each all-reduce is read back
        np.testing.assert_array_equal(V, ref["V"][lo:hi])
        np.testing.assert_array_equal(pi, ref["pi"][lo:hi])


@pytest.mark.parametrize("world,n", [(2, 12), (4, 13), (8, 13), (8, 5)])
def test_device_protocol_uneven_shards_one_host_read(world, n):
    """The device protocol (K / dV stay in int64 tensors, all-reduced in place) over uneven shards,
    including ranks with no grids (8 ranks, 5 grids): equal to one global loop, two all-reduces and
    ONE host read per solve, and the reducer reused across solves."""
    g = load("grids_fourrooms.npz")
    cells = np.stack([cells_from_enc(e) for e in g["enc"][:n]])
    ref = oracle.value_iteration(0, cells)
    out = run_world(cells, world, device_proto=True, solves=2)
    assert len(out) == world
    for rank, (k, nred, V, pi, lo, hi, reads, total_calls, proto) in out.items():
        assert k == ref["sweeps"], (rank, k)
        assert proto is (hi > lo)  # an empty rank drives the same collectives from the host
        assert nred == 1 and reads == 1  # deterministic grids: one all-reduce, one host wait
        assert total_calls == 2  # two solves on one reducer, no agreement collective
        if hi > lo:
            np.testing.assert_array_equal(V, ref["V"][lo:hi])
            np.testing.assert_array_equal(pi, ref["pi"][lo:hi])


@pytest.mark.parametrize("world,n,slip", [(4, 3, None), (8, 5, 0.9), (4, 9, None)])
def test_mixed_protocol_peers(world, n, slip):
    """More ranks than grids (EmptyShards) next to shards that can only run the host protocol, and
    device-capable shards next to host-only ones ("mixed"): each rank takes its own path, and both
    paths issue the same collectives on the same int64 words, so the group never mismatches."""
    g = load("grids_fourrooms.npz")
    cells = np.stack([cells_from_enc(e) for e in g["enc"][:n]])
    ref = oracle.value_iteration(0, cells, slip_p=slip)
    out = run_world(cells, world, slip=slip, device_proto="mixed", solves=2)
    for rank, (k, nred, V, pi, lo, hi, reads, total_calls, proto) in out.items():
        assert k == ref["sweeps"], (rank, k)
        assert proto is (hi > lo and rank % 2 == 0), rank
        assert nred == (1 if slip is None else 2) and total_calls == 2 * nred
        if hi > lo:
            np.testing.assert_array_equal(V, ref["V"][lo:hi])
            np.testing.assert_array_equal(pi, ref["pi"][lo:hi])


@pytest.mark.parametrize("world,n", [(4, 6), (8, 5)])
def test_device_protocol_slip_second_allreduce(world, n):
    """Slip grids end their own rule above an exact fixed point (dV > 0): the device protocol then
    all-reduces dV at K as well -- two all-reduces, two host reads -- and still equals the global loop."""
    g = load("grids_lava11n5.npz")
    cells = np.stack([cells_from_enc(e) for e in g["enc"][:n]])
    ref = oracle.value_iteration(0, cells, slip_p=0.9)
    out = run_world(cells, world, slip=0.9, device_proto=True)
    for rank, (k, nred, V, pi, lo, hi, reads, _, proto) in out.items():
        assert k == ref["sweeps"], (rank, k)
        assert proto is (hi > lo) and nred >= 2 and reads >= 2
        if hi > lo:
            np.testing.assert_array_equal(V, ref["V"][lo:hi])
            np.testing.assert_array_equal(pi, ref["pi"][lo:hi])


@pytest.mark.parametrize("world", [4, 8])
def test_host_protocol_uneven_shards(world):
    g = load("grids_lava11n5.npz")
    cells = np.stack([cells_from_enc(e) for e in g["enc"][:11]])
    ref = oracle.value_iteration(0, cells, slip_p=0.9)
    out = run_world(cells, world, slip=0.9)
    for rank, (k, nred, V, pi, lo, hi, reads, _, _) in out.items():
        assert k == ref["sweeps"]
        np.testing.assert_array_equal(V, ref["V"][lo:hi])
        np.testing.assert_array_equal(pi, ref["pi"][lo:hi])


def test_bits_round_trip_and_order():
    xs = [0.0, 5e-324, 1e-12, 9.99e-7, 1e-6, 0.5, 1.0]
    bits = [double_to_bits(x) for x in xs]
    assert bits == sorted(bits)  # non-negative doubles order like their bits: MAX over bits is MAX
    assert [bits_to_double(b) for b in bits] == xs


class _FakeReducer:
    """One rank's reducer: MAX over one rank is the identity (the proto words stay as written)."""

    def __init__(self):
        import torch

        self.torch = torch
        self.calls = 0
        self.host_reads = 0
        self.wall_s = 0.0
        self.stream = None
        self.device = torch.device("cpu")
        self.proto = torch.zeros(8, dtype=torch.int64)
        self.p_local, self.p_kd, self.p_dv = self.proto[0:4], self.proto[0:2], self.proto[5:6]

    def max(self, x):
        self.calls += 1
        self.host_reads += 1
        return x

    def max_(self, t):
        self.calls += 1


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
    # host path: {K, E} (E unknown: no local_result), dV(K), then 2 fallback sweeps
    assert res["protocol"] == "host" and res["allreduces"] == 4 and res["host_reads"] == 4


def _worker_fresh_empty(rank, world, port, cells, out, solves):
    """Rank 0 passes a NEW EmptyShard to every solve; rank 1 reuses one device-capable shard."""
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    red = Reducer()
    shard = DevOracleShard(cells) if rank == 1 else None
    res = []
    for _ in range(solves):
        r = solve_sharded(shard if rank == 1 else EmptyShard(), reducer=red)
        res.append((r["sweeps"], r["allreduces"], r["protocol"]))
    out[rank] = (res, red.calls, getattr(shard, "V", None))
    dist.barrier()
    dist.destroy_process_group()


def test_fresh_empty_shard_every_solve_next_to_reused_shard():
    """the protocol must not depend on per-rank object state -- a rank building a new
    shard per solve and a rank reusing its shard issue the same collectives on every solve."""
    g = load("grids_fourrooms.npz")
    cells = np.stack([cells_from_enc(e) for e in g["enc"][:4]])
    ref = oracle.value_iteration(0, cells)
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker_fresh_empty, args=(2, port, cells, out, 3), nprocs=2, join=True)
    res0, calls0, _ = out[0]
    res1, calls1, V1 = out[1]
    assert [r[2] for r in res0] == ["host"] * 3 and [r[2] for r in res1] == ["device"] * 3
    assert [r[0] for r in res0] == [r[0] for r in res1] == [ref["sweeps"]] * 3
    assert calls0 == calls1 == 3
    np.testing.assert_array_equal(V1, ref["V"])


_FakeDeviceReducer = _FakeReducer  # the device path uses the same reducer surface


class _NonMonotoneDevShard(_NonMonotoneShard):
    protocol_device = property(lambda self: __import__("torch").device("cpu"))

    def run_local_dev(self, pub):
        pub[0] = self.run_local()
        pub[1] = double_to_bits(5e-7)  # own-rule dV below tol but not an exact fixed point

    def run_to_dev_sync(self, kdv):
        k = int(kdv[0])
        return k, self.run_to(k), bits_to_double(int(kdv[1]))

    def set_result(self, k, dv):
        self.k = k


def test_device_protocol_fallback_loop():
    s = _NonMonotoneDevShard()
    red = _FakeDeviceReducer()
    res = solve_sharded(s, reducer=red)
    assert res["sweeps"] == 5 and res["converged"] and s.final[0] == 5
    # {K, E} and dV(K) all-reduced on the device, then 2 fallback sweeps on the host
    assert res["allreduces"] == 4 and res["host_reads"] == 4


class _BrokenFixedPointShard(_NonMonotoneDevShard):
    """Claims an exact fixed point at its own stop, yet dV at K is not 0: the protocol must refuse."""

    def run_local_dev(self, pub):
        pub[0] = self.run_local()
        pub[1] = 0


def test_device_protocol_refuses_broken_fixed_point():
    with pytest.raises(RuntimeError, match="fixed-point invariant"):
        solve_sharded(_BrokenFixedPointShard(), reducer=_FakeDeviceReducer())


# -- the library's own collectives (LibComm + mgdp_vi_solve_sharded), protocol logic on gloo ---------
class GlooLibComm:
    """LibComm's interface (allreduce_max of int64 host words, an all-reduce counter) over gloo."""

    def __init__(self):
        self.allreduces = 0
        self.host_waits = 0  # as mgdp_comm_host_waits: one per host-driven all-reduce (+ the C path's own)

    def allreduce_max(self, vals):
        import torch
        import torch.distributed as dist

        t = torch.tensor([int(v) for v in vals], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        self.allreduces += 1
        self.host_waits += 1
        return [int(x) for x in t.tolist()]


class LibOracleShard(OracleShard):
    """A shard on the C path: solve_sharded(comm) issues exactly mgdp_vi_solve_sharded's collectives
    (csrc/vi.hip): {K, own-rule dV bits}; dV(K) only if the all-reduced dV bits are non-zero; one
    word per rounding-level fallback sweep."""

    sharded_capable = True

    def solve_sharded(self, comm):
        self.reset()
        k_loc = self.run_local()
        K, e_bits = comm.allreduce_max([k_loc, double_to_bits(self._local[1])])
        comm.host_waits -= 1  # the C path's {K, E} all-reduce stays on the stream ...
        dv = self.run_to(K)
        comm.host_waits += 1  # ... and its one host wait is run_to's result
        if bits_to_double(e_bits) != 0.0:
            dv = bits_to_double(comm.allreduce_max([double_to_bits(dv)])[0])
        k = K
        while not (dv < self.tol) and k < self.max_sweeps:
            dv = bits_to_double(comm.allreduce_max([double_to_bits(self.sweep())])[0])
            k += 1
        self.finish(k, dv)
        self.dv, self.converged = dv, dv < self.tol
        return k


def _lib_worker(rank, world, port, cells, slip, out, kinds):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(len(cells), rank, world)
    comm = GlooLibComm()
    kind = kinds[rank % len(kinds)]
    shard = EmptyShard() if hi == lo else (LibOracleShard if kind == "lib" else OracleShard)(cells[lo:hi], slip=slip)
    res = solve_sharded(shard, comm=comm)
    out[rank] = (res["sweeps"], res["allreduces"], getattr(shard, "V", None), getattr(shard, "pi", None), lo, hi,
                 res["protocol"], res["host_reads"])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("slip", [None, 0.9])
@pytest.mark.parametrize("world,kinds", [(2, ("lib",)), (2, ("lib", "host")), (4, ("host", "lib")), (8, ("lib",))])
def test_lib_comm_protocol_matches_global_loop(world, kinds, slip):
    """Ranks on mgdp_vi_solve_sharded's collective sequence, host-driven peers and empty shards (8
    ranks, 6 grids) meet in the same collectives; the result is one global Jacobi loop's."""
    g = load("grids_fourrooms.npz")
    cells = np.stack([cells_from_enc(e) for e in g["enc"][:6 if world == 8 else 10]])
    ref = oracle.value_iteration(0, cells, slip_p=slip, dtype="f64")
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_lib_worker, args=(world, port, cells, slip, out, kinds), nprocs=world, join=True)
    res = dict(out)
    for r, (k, n, V, pi, lo, hi, proto, waits) in res.items():
        assert k == ref["sweeps"]
        # deterministic: one collective per solve; slip: the dV(K) word too
        assert n == (1 if slip is None else 2) or (slip is not None and n >= 2)
        # host waits: every collective of a host-driven rank; on the C path the {K, E} all-reduce stays on
        # the stream and run_to's result is the wait instead -- so the count equals the collectives either way
        assert waits == n
        assert proto == ("lib" if (hi > lo and kinds[r % len(kinds)] == "lib") else "lib-host")
        if hi > lo:
            np.testing.assert_array_equal(V, ref["V"][lo:hi])
            np.testing.assert_array_equal(pi, ref["pi"][lo:hi])
