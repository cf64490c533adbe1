"""Host-side cost of each step of the sharded device protocol (distributed._device_protocol) over a
one-rank RCCL group: the shard of an 8-way split of LavaS11N5 x 65536 solved N times, each step
timed with perf_counter (medians in us).  Run as a single process with WORLD_SIZE=1 RANK=0
MASTER_ADDR=127.0.0.1 MASTER_PORT=... in the environment."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.distributed as dist

    import minigrid_dynamicprogramming_amd as mg
    from minigrid_dynamicprogramming_amd import _lib, gen
    from minigrid_dynamicprogramming_amd.distributed import Reducer, solve_sharded

    _lib.pin_host_thread(0)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    cells = gen.generate("MiniGrid-LavaCrossingS11N5-v0", 0, 8192, enc=False, cells=True, agent=False)["cells"]
    vi = mg.ValueIteration(cells, dtype="f32")
    red = Reducer()
    for _ in range(20):
        solve_sharded(vi, reducer=red)
    torch.cuda.synchronize()
    n = 200
    t = np.zeros((n, 8))
    for i in range(n):
        a = time.perf_counter()
        vi.bind_stream(red.stream_ptr)
        prev = red.enter_stream()
        b = time.perf_counter()
        vi.reset()
        c = time.perf_counter()
        vi.run_local_dev(red.p_local)
        d = time.perf_counter()
        red.max_(red.p_kd)
        e = time.perf_counter()
        k, dv, rule = vi.run_to_dev_sync(red.p_kd)
        f = time.perf_counter()
        vi.set_result(k, dv)
        red.exit_stream(prev)
        g = time.perf_counter()
        vi.finish(k, dv)
        h = time.perf_counter()
        t[i] = [b - a, c - b, d - c, e - d, f - e, g - f, h - g, h - a]
    med = np.median(t, axis=0) * 1e6
    names = ["bind+stream_ctx", "reset", "run_local_dev", "all_reduce_call", "run_to_dev_sync(wait)",
             "set_result+ctx_exit", "finish", "total"]
    out = {k: round(float(v), 2) for k, v in zip(names, med)}
    ts = []
    for _ in range(n):
        a = time.perf_counter()
        solve_sharded(vi, reducer=red)
        ts.append(time.perf_counter() - a)
    out["solve_sharded_us"] = round(float(np.median(ts)) * 1e6, 2)
    ts = []
    for _ in range(n):
        a = time.perf_counter()
        vi.solve()
        ts.append(time.perf_counter() - a)
    out["direct_solve_us"] = round(float(np.median(ts)) * 1e6, 2)
    # the host cost of the two steps made cheaper in round 4, old way beside new way
    def med(f):
        ts = []
        for _ in range(n):
            a = time.perf_counter()
            f()
            ts.append(time.perf_counter() - a)
        return round(float(np.median(ts)) * 1e6, 2)

    def ctx():
        with torch.cuda.stream(red.stream):
            pass

    out["torch_stream_ctx_us"] = med(ctx)
    out["enter_exit_stream_us"] = med(lambda: red.exit_stream(red.enter_stream()))
    out["dist_all_reduce_us"] = med(lambda: dist.all_reduce(red.p_kd, op=dist.ReduceOp.MAX))
    out["pg_allreduce_us"] = med(lambda: red._all_reduce_max(red.p_kd))
    torch.cuda.synchronize()
    print(json.dumps(out), flush=True)
    vi.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
