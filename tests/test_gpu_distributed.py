"""Sharded value iteration on the GPU: two ranks (gloo control plane) share one MI355X, each rank
solving its shard through libmgdp; the result must equal a single-device solve of the whole batch
(the same global stopping sweep, V and pi bit for bit)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cells, kw, out):
    import torch.distributed as dist

    import minigrid_dynamicprogramming_amd as mg
    from minigrid_dynamicprogramming_amd.distributed import shard_range, solve_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(len(cells), rank, world)
    vi = mg.ValueIteration(cells[lo:hi], **kw)
    res = solve_sharded(vi)
    out[rank] = (res["sweeps"], res["allreduces"], vi.values(), vi.policy(), lo, hi)
    vi.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("method", ["fused", "sweep"])
@pytest.mark.parametrize("env_id,slip", [("MiniGrid-FourRooms-v0", None), ("MiniGrid-LavaCrossingS11N5-v0", 0.9),
                                         ("MiniGrid-DoorKey-8x8-v0", None)])
def test_two_ranks_match_single_device(env_id, slip, method):
    import minigrid_dynamicprogramming_amd as mg

    env = mg.make(env_id)
    encs = np.stack([env.generate(seed=s)[0] for s in range(96)])
    kw = dict(dtype="f32", method=method, slip_p=slip)
    ref = mg.value_iteration(encs, **kw)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _port(), encs, kw, out), nprocs=2, join=True)
    for rank, (k, nred, V, pi, lo, hi) in dict(out).items():
        assert k == ref.sweeps
        # gloo with GPU handles: the host protocol.  Deterministic grids end their own rule at an
        # exact fixed point: one all-reduce of {K, own-rule dV}; slip grids also all-reduce dV at K
        assert nred == 1 if slip is None else nred >= 2
        np.testing.assert_array_equal(V, ref.V[lo:hi])
        np.testing.assert_array_equal(pi, ref.pi[lo:hi])


_DEVICE_PROTO = r"""
import os, sys
import torch  # first: PyTorch-ROCm and libmgdp share libamdhip64.so.7, the first one loaded serves both
import numpy as np
sys.path.insert(0, sys.argv[1])
import minigrid_dynamicprogramming_amd as mg
from minigrid_dynamicprogramming_amd import gen
from minigrid_dynamicprogramming_amd.distributed import Reducer, bits_to_double, solve_sharded

mode = sys.argv[2]
env_id, B, dtype = sys.argv[3], int(sys.argv[4]), sys.argv[5]
slip = float(sys.argv[6]) if len(sys.argv) > 6 else None
cells = gen.generate(env_id, 0, B, enc=False, cells=True, agent=False)["cells"]
# the reference is the CPU oracle's literal global Jacobi loop over the whole batch (tests only)
from oracle import oracle
o = oracle.value_iteration(1 if "DoorKey" in env_id else 0, cells, slip_p=slip, dtype=dtype, nthreads=8)
k_ref, V_ref, pi_ref = o["sweeps"], o["V"], o["pi"]
vi = mg.ValueIteration(cells, dtype=dtype, slip_p=slip)
if mode == "steps":
    # the C entry points alone, on a torch stream: K and dV stay in device memory between launches
    s = torch.cuda.Stream()
    vi.bind_stream(s.cuda_stream)
    p = torch.zeros(8, dtype=torch.int64, device="cuda")
    with torch.cuda.stream(s):
        for rep in range(3):
            vi.reset()
            vi.run_local_dev(p[0:4])
            vi.run_to_dev(p[0:1], p[4:8])
            h = p.tolist()
            k, dv = h[0], bits_to_double(h[5])
            assert k == k_ref and h[4] == k and h[6] == k and dv < 1e-6, (h, k_ref)
            vi.set_result(k, dv)
            vi.finish(k, dv)
            assert np.array_equal(vi.values(), V_ref) and np.array_equal(vi.policy(), pi_ref)
elif mode == "sync":
    # run_local_dev, then run_to_dev_sync: K read on the device, the result and p[1] (the own-rule
    # dV; all-reduced in a real run) come back through host-mapped words, no stream synchronisation
    s = torch.cuda.Stream()
    vi.bind_stream(s.cuda_stream)
    p = torch.zeros(8, dtype=torch.int64, device="cuda")
    with torch.cuda.stream(s):
        for rep in range(3):
            vi.reset()
            vi.run_local_dev(p[0:4])
            k, dv, rule = vi.run_to_dev_sync(p[0:2])
            # deterministic grids end their own rule at an exact fixed point: own-rule dV and dV(K) are 0
            assert k == k_ref and dv == 0.0 and rule == 0.0, (k, dv, rule, k_ref)
            assert vi.local_result()[0] == k
            vi.set_result(k, dv)
            vi.finish(k, dv)
            assert np.array_equal(vi.values(), V_ref) and np.array_equal(vi.policy(), pi_ref)
elif mode == "lib1":
    # the library's own communicator (mgdp_comm_*: RCCL from libmgdp, one rank), bootstrapped over a
    # one-rank gloo group; one mgdp_vi_solve_sharded call per solve
    import torch.distributed as dist
    from minigrid_dynamicprogramming_amd.distributed import LibComm
    dist.init_process_group("gloo")
    comm = LibComm()
    for rep in range(3):
        res = solve_sharded(vi, comm=comm)
        assert res["protocol"] == "lib", res
        if slip is None:
            assert res["sweeps"] == k_ref and res["allreduces"] == 1, res
        else:
            assert res["sweeps"] == k_ref and res["allreduces"] >= 2, res
        assert np.array_equal(vi.values(), V_ref) and np.array_equal(vi.policy(), pi_ref)
    # a rank whose handle cannot run the C path (the sweep method) joins host-driven
    hs = mg.ValueIteration(cells, dtype=dtype, slip_p=slip, method="sweep")
    res = solve_sharded(hs, comm=comm)
    assert res["protocol"] == "lib-host" and res["sweeps"] == k_ref, res
    assert np.array_equal(hs.values(), V_ref) and np.array_equal(hs.policy(), pi_ref)
    hs.close()
    comm.close()
    dist.destroy_process_group()
else:
    import torch.distributed as dist
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))  # RCCL, one rank
    red = Reducer(timing=True)
    for rep in range(3):
        res = solve_sharded(vi, reducer=red)
        # deterministic grids: one all-reduce of {K, own-rule dV} and one host wait per solve; slip
        # grids also all-reduce dV at K
        if slip is None:
            assert res["sweeps"] == k_ref and res["allreduces"] == 1 and res["host_reads"] == 1, res
        else:
            assert res["sweeps"] == k_ref and res["allreduces"] >= 2 and res["host_reads"] >= 2, res
        assert np.array_equal(vi.values(), V_ref) and np.array_equal(vi.policy(), pi_ref)
    torch.cuda.synchronize()
    print("allreduce device ms", red.collect(), "calls", red.calls)
    dist.destroy_process_group()
vi.close()
print("device protocol ok")
"""


@pytest.mark.parametrize("mode", ["steps", "sync", "rccl1", "lib1"])
@pytest.mark.parametrize("env_id,B,dtype", [("MiniGrid-LavaCrossingS11N5-v0", 2048, "f32"),
                                            ("MiniGrid-FourRooms-v0", 300, "f64"),
                                            ("MiniGrid-DoorKey-16x16-v0", 700, "f32"),
                                            ("MiniGrid-Empty-16x16-v0", 1, "f32")])
def test_device_protocol(mode, env_id, B, dtype):
    """mgdp_vi_run_local_dev / run_to_dev / set_result: K and dV in a device buffer, read once.
    "steps": the entry points on a torch stream; "sync": run_local_dev + run_to_dev_sync (result via
    host-mapped words); "rccl1": distributed.solve_sharded over a one-rank
    RCCL group (the all-reduces are real RCCL collectives ordered on the protocol stream); "lib1":
    the library's own RCCL communicator (mgdp_vi_solve_sharded, one C call per solve) plus a
    sweep-method handle joining its collectives host-driven.  Batches
    on both sides of the in-kernel-reduce limit (512) and a lone grid; every mode equal to the CPU
    oracle's global loop (sweeps, V, pi bit for bit)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-c", _DEVICE_PROTO, root, mode, env_id, str(B), dtype], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0 and "device protocol ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("mode", ["rccl1", "lib1"])
@pytest.mark.parametrize("B", [300, 2048])
def test_device_protocol_rccl1_slip(B, mode):
    """Slip grids over a one-rank RCCL group: the own-rule dV is not an exact fixed point, so the
    protocol all-reduces dV at K too (two collectives) and still equals the oracle's global loop."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-c", _DEVICE_PROTO, root, mode, "MiniGrid-LavaCrossingS11N5-v0", str(B),
                        "f32", "0.9"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "device protocol ok" in r.stdout, r.stdout + r.stderr


# -- mgdp_vi_solve_sharded at world > 1 on one GPU: the host communicator -----------------------------
def _multi_worker(rank, world, port, env_id, B, dtype, slip, kinds, out):
    """One rank: a gloo group for the bootstrap, the library's host communicator (mgdp_comm_create_host),
    and this rank's shard on the path its kind names: "lib" = a fused handle, one mgdp_vi_solve_sharded
    call per solve (the C code's collectives); "host" = a sweep-method handle driving the same
    collectives from Python (mgdp_comm_allreduce_max); "empty" = no grids (EmptyShard)."""
    import torch.distributed as dist

    import minigrid_dynamicprogramming_amd as mg
    from minigrid_dynamicprogramming_amd import gen
    from minigrid_dynamicprogramming_amd.distributed import EmptyShard, LibComm, shard_range, solve_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    kind = kinds[rank]
    holders = [r for r in range(world) if kinds[r] != "empty"]
    lo = hi = 0
    if kind != "empty":
        lo, hi = shard_range(B, holders.index(rank), len(holders))
    cells = gen.generate(env_id, 0, B, enc=False, cells=True, agent=False)["cells"]
    comm = LibComm(kind="host", device=0)
    if kind == "empty":
        shard = EmptyShard()
    else:
        shard = mg.ValueIteration(cells[lo:hi], dtype=dtype, slip_p=slip, method="fused" if kind == "lib" else "sweep")
    res = []
    for _ in range(2):  # a second solve on the same communicator and handles
        r = solve_sharded(shard, comm=comm)
        res.append((r["sweeps"], r["allreduces"], r["host_reads"], r["protocol"]))
    V = shard.values() if kind != "empty" else None
    pi = shard.policy() if kind != "empty" else None
    out[rank] = (res, V, pi, lo, hi, comm.kind)
    if kind != "empty":
        shard.close()
    comm.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("env_id,B,dtype,slip,kinds", [
    ("MiniGrid-FourRooms-v0", 96, "f32", None, ("lib", "lib")),
    ("MiniGrid-FourRooms-v0", 96, "f32", None, ("lib", "host")),
    ("MiniGrid-LavaCrossingS11N5-v0", 600, "f32", 0.9, ("lib", "lib")),
    ("MiniGrid-LavaCrossingS11N5-v0", 600, "f32", 0.9, ("host", "lib")),
    ("MiniGrid-LavaCrossingS11N5-v0", 2048, "f32", None, ("lib", "host", "empty", "lib")),
    ("MiniGrid-FourRooms-v0", 300, "f64", 0.9, ("lib", "empty", "lib", "host")),
    ("MiniGrid-DoorKey-16x16-v0", 64, "f32", None, ("lib", "lib", "lib", "lib")),
])
def test_solve_sharded_multi_rank_host_comm(env_id, B, dtype, slip, kinds):
    """The unchanged C entry mgdp_vi_solve_sharded at world 2 and 4 on one GPU (RCCL refuses two ranks
    on one device, so the ranks share the host communicator): fused ranks on the C path next to
    host-driven sweep-method ranks and empty shards, deterministic and slip grids.  Every rank ends at
    the oracle's global stopping sweep with its block's V and pi bit for bit, and every rank issues
    the same collectives: 1 per deterministic solve, >= 2 for slip (the dV(K) word), equal on all ranks
    (the C sequence is the Python restatement's)."""
    from oracle import oracle
    from minigrid_dynamicprogramming_amd import gen

    cells = gen.generate(env_id, 0, B, enc=False, cells=True, agent=False)["cells"]
    o = oracle.value_iteration(1 if "DoorKey" in env_id else 0, cells, slip_p=slip, dtype=dtype, nthreads=8)
    world = len(kinds)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_multi_worker, args=(world, _port(), env_id, B, dtype, slip, kinds, out), nprocs=world, join=True)
    got = dict(out)
    assert sorted(got) == list(range(world))
    counts = set()
    for rank, (res, V, pi, lo, hi, ckind) in got.items():
        assert ckind == "host"  # the host communicator
        for k, nred, nwait, proto in res:
            assert k == o["sweeps"], (rank, k, o["sweeps"])
            assert proto == ("lib" if kinds[rank] == "lib" else "lib-host"), (rank, proto)
            assert nred == 1 if slip is None else nred >= 2
            assert nwait >= 1
            counts.add(nred)
        if kinds[rank] != "empty":
            np.testing.assert_array_equal(V, o["V"][lo:hi])
            np.testing.assert_array_equal(pi, o["pi"][lo:hi])
    assert len(counts) == 1, counts  # every rank met the same collectives
