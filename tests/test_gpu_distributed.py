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
        assert nred >= 2
        np.testing.assert_array_equal(V, ref.V[lo:hi])
        np.testing.assert_array_equal(pi, ref.pi[lo:hi])
