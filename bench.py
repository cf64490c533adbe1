#!/usr/bin/env python3
"""Benchmark: state-action Bellman updates/s + sweeps-to-converge (BASELINE.json metric).

One "step" = one complete value-iteration solve of the workload on every rank: V_0 = 0, Jacobi
sweeps until the global rule max|V_k - V_{k-1}| < tol (gamma = 0.99, tol = 1e-6), policy
extraction, sweep count returned to the host.  Inputs (grid cells) are resident in HBM before the
timed region.  value = (sum over ranks of B_r * S * A * sweeps) * steps / max-over-ranks time.

Workloads; default = BASELINE configs[1]:
  empty16        MiniGrid-Empty-16x16-v0, 1 grid per GPU (N > 1: replicas only)
  empty16x65536  Empty-16x16 x 65536 replicas per GPU (SURVEY 8(d) "R", the HBM-roofline sizing)
  fourrooms4096  MiniGrid-FourRooms-v0, 4096 seeds per GPU
  lava65536      MiniGrid-LavaCrossingS11N5-v0, 65536 seeds sharded over N GPUs (RCCL dV all-reduce)
  doorkey65536   MiniGrid-DoorKey-16x16-v0 (pos, dir, has_key, door_open), 65536 seeds sharded

Side paths (measured to the same bar; their own metric, not the headline):
  step_doorkey16x65536 / step_fourrooms65536 / step_lava65536
                 batched MiniGridEnv.step + gen_obs (csrc/envs.hip), 65536 envs per GPU, env-steps/s
  gen_lava65536 / gen_fourrooms65536 / gen_doorkey16x65536
                 batched reset(seed) grid generation (csrc/gen.hip), 65536 seeds per GPU, grids/s

Run:  python bench.py [--gpus N --steps K --warmup W --workload NAME --method fused|sweep ...]
      N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N, or plain
      `python bench.py --gpus N`, which starts the N ranks itself (torch.distributed.run as a child
      process, before any GPU call) and exits with its status.
The line of the default workload also carries a "batched" block for BASELINE config 3
(fourrooms4096, independent per GPU) and a "sharded" block per BASELINE multi-GPU config
(lava65536, doorkey65536): the global batch sharded over the N ranks (at N = 1 the direct solve),
updates/s over the whole job, ms per solve, sweeps, at N > 1 the collectives per solve, and at
N = 1 the oracle timed on a bounded sample of the same grids (1 thread and all cores).  These
blocks run before the headline, whose resident server is primed to a stated steady state.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "state-action Bellman updates/sec + DP sweeps-to-converge, Empty-16x16"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: HBM3E 8.0 TB/s peak

WORKLOADS = {
    "empty16": dict(env_id="MiniGrid-Empty-16x16-v0", per_gpu=1, replicate=True, sharded=False),
    # a stream of distinct lone grids: every step solves the next of 64 FourRooms seeds, handed to the
    # resident server from HBM with the request (mgdp_vi_load_cells_device), no drain or relaunch
    "fourrooms1": dict(env_id="MiniGrid-FourRooms-v0", per_gpu=1, distinct=64, replicate=False, sharded=False),
    "empty16x65536": dict(env_id="MiniGrid-Empty-16x16-v0", per_gpu=65536, replicate=True, sharded=False),
    "fourrooms4096": dict(env_id="MiniGrid-FourRooms-v0", per_gpu=4096, replicate=False, sharded=False),
    "lava65536": dict(env_id="MiniGrid-LavaCrossingS11N5-v0", global_grids=65536, replicate=False, sharded=True),
    "doorkey65536": dict(env_id="MiniGrid-DoorKey-16x16-v0", global_grids=65536, replicate=False, sharded=True),
}


STEP_WORKLOADS = {
    "step_doorkey16x65536": dict(env_id="MiniGrid-DoorKey-16x16-v0", per_gpu=65536),
    "step_fourrooms65536": dict(env_id="MiniGrid-FourRooms-v0", per_gpu=65536),
    "step_lava65536": dict(env_id="MiniGrid-LavaCrossingS11N5-v0", per_gpu=65536),
    # 2^20 DoorKey-16 envs: ~390 MB of env state + obs per step, past the 256 MB MALL (HBM-bound sizing)
    "step_doorkey16x1m": dict(env_id="MiniGrid-DoorKey-16x16-v0", per_gpu=1 << 20),
}
GEN_WORKLOADS = {
    "gen_lava65536": dict(env_id="MiniGrid-LavaCrossingS11N5-v0", per_gpu=65536),
    "gen_fourrooms65536": dict(env_id="MiniGrid-FourRooms-v0", per_gpu=65536),
    "gen_doorkey16x65536": dict(env_id="MiniGrid-DoorKey-16x16-v0", per_gpu=65536),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def step_bytes_per_env_step(view: int) -> int:
    """Algorithmic HBM bytes of one env step (csrc/envs.hip layout): reads action 4, agent
    (x, y, dir, step_count) 16, carry 8, max_steps 4, see_through 1 and the view window's
    view*view cells x 3 planes; writes the obs view*view*3, direction 4, reward 8, terminated 1,
    truncated 1, status 4, agent 16, carry 8 (pickup/drop/toggle cell writes are rare, not counted)."""
    vv3 = view * view * 3
    return (4 + 16 + 8 + 4 + 1 + vv3) + (vv3 + 4 + 8 + 1 + 1 + 4 + 16 + 8)


def algorithmic_bytes_per_update(tsize: int, A: int) -> float:
    """read V'[s'] (sizeof V) + 1 B cell type + write V[s] amortised over A."""
    return tsize + 1 + tsize / A


def compulsory_bytes_per_sweep(S: int, HW: int, tsize: int) -> int:
    """2*S*sizeof(V) + W*H per grid-sweep (read V once, write V once, read cells)."""
    return 2 * S * tsize + HW


def shard_of(world: int) -> int:
    """How many ways a sharded workload's global batch is split: the world size, or at world 1 the
    MGDP_BENCH_SHARD_OF=N rehearsal knob (never set by the driver), which makes the one rank solve
    rank 0's shard of an N-way split -- the per-rank work of an N-GPU run, measured on one GPU."""
    n = int(os.environ.get("MGDP_BENCH_SHARD_OF", "0") or 0)
    return n if world == 1 and n > 1 else world


def make_cells(spec, rank, world, seed_offset=0):
    """This rank's grids of a workload; seed_offset shifts every seed (fresh grid sets)."""
    from minigrid_dynamicprogramming_amd import make
    from minigrid_dynamicprogramming_amd.distributed import shard_range

    env = make(spec["env_id"])
    if spec.get("sharded"):
        lo, hi = shard_range(spec["global_grids"], rank, shard_of(world))
    elif spec.get("distinct"):
        lo, hi = rank * spec["distinct"], (rank + 1) * spec["distinct"]
    else:
        lo, hi = rank * spec["per_gpu"], (rank + 1) * spec["per_gpu"]
    if spec.get("replicate"):
        enc, _ = env.generate(seed=0)
        one = np.ascontiguousarray(enc[..., 0].T)
        return np.broadcast_to(one, (hi - lo,) + one.shape).copy(), (lo, hi)
    # reset(seed) for every seed of this rank's shard, generated on the GPU (csrc/gen.hip; pinned
    # to the reference's grid digests by tests/test_gpu_gen.py); not part of the timed region
    from minigrid_dynamicprogramming_amd import gen

    cells = gen.generate(env, lo + seed_offset, hi - lo, enc=False, cells=True, agent=False)["cells"]
    return cells, (lo, hi)


def cpu_baseline(cells, model, gamma, tol, dtype, budget_s=8.0, nthreads=1, lone=False, fixed_point=False):
    """Time the oracle (oracle/, a C restatement of the same algorithm) on a bounded sample.
    lone: the workload solves its grids one at a time (each its own stopping sweep).
    fixed_point: orc_vi_fp, the literal loop with the GPU's per-grid fixed-point stop (a grid whose
    sweep changed nothing is not swept again; same K, V, pi) -- the like-for-like CPU leg of a
    batched config; updates are still counted as B*S*A*K, as the metric defines them."""
    import threading

    from oracle import oracle

    model_id = 0 if model == "xyd" else 1
    # 32 grids per thread (a threaded batch solve needs work for every thread), 32 for one thread
    sample = cells[: min(len(cells), 32 * max(1, nthreads))]
    S = sample.shape[1] * sample.shape[2] * (4 if model_id == 0 else 16)
    A = 7 if model_id == 0 else 5
    # A lone-grid workload gives each OpenMP thread 64 states per sweep, so a threaded solve times
    # fork/join, not the cores: run one independent single-threaded solve loop per thread instead
    # (ctypes drops the GIL inside the oracle call).
    replicated = nthreads > 1 and (len(sample) < nthreads or lone)
    loops = nthreads if replicated else 1
    per_call = 1 if replicated else nthreads
    counts = [[0, 0, 0] for _ in range(loops)]  # updates, solves, sweeps
    t0 = time.perf_counter()

    def loop(c):
        i = 0
        while True:
            g = sample[i % len(sample)][None] if lone else sample
            i += 1
            r = oracle.value_iteration(model_id, g, gamma, tol, dtype=dtype, nthreads=per_call, fixed_point=fixed_point)
            c[0] += len(g) * S * A * r["sweeps"]
            c[1] += 1
            c[2] = r["sweeps"]
            if time.perf_counter() - t0 >= budget_s:
                break

    if loops == 1:
        loop(counts[0])
    else:
        ts = [threading.Thread(target=loop, args=(c,)) for c in counts]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    el = time.perf_counter() - t0
    updates = sum(c[0] for c in counts)
    solves = sum(c[1] for c in counts)
    how = f", {loops} threads each solving its own replica" if replicated else ""
    what = (f"{solves} lone-grid solves cycling over {len(sample)} distinct grids" if lone else
            f"{solves} full solves of {len(sample)} grid(s)")
    fn = "orc_vi_fp (per-grid fixed-point stop)" if fixed_point else "orc_vi (literal global loop)"
    return {"value": updates / el, "unit": "updates/s", "cores": nthreads, "kind": "port",
            "sample": f"{what} of the same workload ({counts[0][2]} sweeps in the last, {dtype}{how}), "
                      f"oracle/mgdp_oracle.c {fn}, {el:.1f} s"}


def load_traffic(key, solves_per_launch, grids=None):
    """HBM bytes per launch from the committed PMC passes (tools/pmc_traffic.sh).  A persistent
    server launch serves many solves: its entry is per solve, scaled to this launch's solves.  A
    batched entry was measured on `grids_per_launch` grids: a rank launching `grids` of them (a
    shard of the global batch) moves grids / grids_per_launch of those bytes (None when the entry
    does not say how many grids it measured)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        d = json.load(f)
    v = d.get(key)
    if v is None:
        return None
    if "bytes_per_solve" in v:
        return v["bytes_per_solve"] * solves_per_launch
    b = v.get("bytes_per_launch")
    measured = v.get("grids_per_launch")
    if grids is not None and b is not None:
        if not measured:
            return None
        b = b * grids / measured
    return b


def self_launch(argv) -> int:
    """`--gpus N > 1` without a torch.distributed environment: start the N ranks as a child
    `torch.distributed.run` (one process per GPU, rendezvous on 127.0.0.1) -- before this process
    touches the GPU, and never as an exec -- and return its exit status (non-zero if any rank
    failed).  Rank 0's JSON line reaches stdout through the inherited file descriptor."""
    import socket
    import subprocess

    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    n = ap.parse_known_args(argv)[0].gpus
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]
    log(f"bench: --gpus {n} without WORLD_SIZE: launching {n} ranks: {' '.join(cmd)}")
    return subprocess.run(cmd).returncode


def dry_run(args, rank, world):
    """MGDP_BENCH_DRYRUN=1 (tests/test_bench_launch.py, CPU only): the rank plumbing of a multi-GPU
    run without a GPU -- gloo group, barrier, max-over-ranks of a fake region, rank 0's line.
    MGDP_BENCH_DRYRUN_FAIL_RANK=r makes rank r fail, to check the launcher's exit status."""
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")
    if int(os.environ.get("MGDP_BENCH_DRYRUN_FAIL_RANK", "-1")) == rank:
        log(f"[rank {rank}] dry run: failing on purpose")
        sys.exit(3)
    t = torch.tensor([0.001 * (rank + 1)], dtype=torch.float64)
    if world > 1:
        dist.barrier()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "dry_run": True, "elapsed_max": float(t.item()),
                          "ranks": [int(os.environ.get("RANK", "0")), world]}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def workload_roofline(args, dtype, m, workload, grids):
    """The roofline object of a measured workload: SURVEY 8(d) algorithmic bytes per launch / the
    dominant kernel's average launch time (HIP events), compulsory bytes, and the committed PMC
    traffic scaled to this rank's `grids`."""
    vi_info = m["info"]
    A = vi_info["A"]
    tsize = 4 if dtype == "f32" else 8
    bpu = algorithmic_bytes_per_update(tsize, A)
    launches = m["launches"]
    avg_launch_s = (m["kern_ms"] / 1000.0) / max(launches, 1)
    # solves inside the timed launches: the K timed solves plus the priming solves a resident
    # server's launch also spans
    solves_in_launches = args.steps + m["timed_primed"]  # the timed launches: relaunch priming + region
    # algorithmic bytes of the work EXECUTED: with fixed-point completion a grid at an exact fixed
    # point is not swept past its own stop, so the batched launches run mean_grid_sweeps per grid, not K
    ex = m.get("executed")
    swept = ex["mean_grid_sweeps"] if ex else float(np.mean(m["sweeps"]))
    upd_per_solve = float(vi_info["updates_per_sweep"]) * float(swept)
    alg_bytes_launch = upd_per_solve * solves_in_launches * bpu / max(launches, 1)
    achieved = alg_bytes_launch / avg_launch_s / 1e9 if launches else 0.0
    comp_launch = compulsory_bytes_per_solve(vi_info, tsize, args.method, m["sweeps"][-1]) * solves_in_launches / max(launches, 1)
    key = f"{workload}/{args.method}/{args.mapping}/{dtype}"
    traffic = load_traffic(key, solves_in_launches / max(launches, 1), grids=None if vi_info["persistent"] else grids)
    roofline = {
        "bound": "hbm", "kernel": vi_info["kernel"],
        "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
        "traffic": traffic, "launches": launches, "avg_launch_us": avg_launch_s * 1e6,
        "alg_bytes_per_launch": alg_bytes_launch, "alg_bytes_per_update": bpu,
        "solves_per_launch": solves_in_launches / max(launches, 1),
        "compulsory_bytes_per_launch": comp_launch,
        "compulsory_frac": comp_launch / max(avg_launch_s, 1e-30) / 1e9 / HBM_PEAK_GBS,
        "basis": "executed updates (grid-sweeps run)" if ex else "B*S*A*K",
        "note": ("achieved = SURVEY 8(d) algorithmic bytes (sizeof V + 1 + sizeof V / A per executed (s,a) update) "
                 "per launch / the launch's HIP-event duration; compulsory = the bytes this kernel must move per launch "
                 "(fused/served: cells in + V and pi out once per solve, spread over the solve's launches; sweep: "
                 "2*S*sizeof V + W*H per grid-sweep); traffic = PMC HBM bytes per launch (profiles/pmc_traffic.json), "
                 "scaled to this rank's grids"),
    }
    sq = load_sq(f"{key}/{vi_info['kernel']}")
    if sq and sq.get("valu_insts_per_launch") and launches and not vi_info["persistent"]:
        # the batched fused kernel keeps V in LDS: its limits are issue / LDS / latency, not HBM
        scale = grids / sq["grids_per_launch"] if sq.get("grids_per_launch") else 1.0
        lane_ops = sq["valu_insts_per_launch"] * scale * 64.0 / avg_launch_s
        roofline["valu"] = {"achieved": lane_ops, "peak": VALU_PEAK_LANE_OPS, "unit": "lane-ops/s",
                            "frac": lane_ops / VALU_PEAK_LANE_OPS, "lds_array_busy": sq.get("lds_array_busy"),
                            "wave_split": sq.get("wave_split"), "source": sq.get("source"),
                            "work": "executed VALU instructions (PMC SQ_INSTS_VALU), not B*S*A*K"}
    if workload == "empty16":
        roofline["regime"] = ("single 4 KiB V grid on one resident workgroup: latency bound (barrier + LDS round trip "
                              "per sweep, host hand-off per solve); HBM is not the limit here (SURVEY 8(d) "
                              "caveats); see roofline_hbm for the kernels at the HBM-sized config R")
    if vi_info["persistent"]:
        roofline["launch_note"] = ("lone grid: one resident vi_serve_kernel launch serves the priming solves and every "
                                   "timed solve (host posts a request word, the workgroup solves and publishes), so "
                                   "its duration spans the timed region")
    if roofline["frac"] > 1.0:  # LDS-served gathers: the algorithmic figure is not an HBM rate
        roofline["alg_equiv_gbs"] = achieved
        meas = traffic if traffic else comp_launch
        roofline["achieved"] = meas / avg_launch_s / 1e9
        roofline["frac"] = roofline["achieved"] / HBM_PEAK_GBS
        roofline["achieved_basis"] = "pmc traffic" if traffic else "compulsory bytes"
    return roofline


def main():
    if int(os.environ.get("WORLD_SIZE", "0") or 0) == 0:
        ap0 = argparse.ArgumentParser(add_help=False)
        ap0.add_argument("--gpus", type=int, default=1)
        if ap0.parse_known_args()[0].gpus > 1:
            sys.exit(self_launch(sys.argv[1:]))

    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--workload", default="empty16", choices=sorted(WORKLOADS) + sorted(STEP_WORKLOADS) + sorted(GEN_WORKLOADS))
    ap.add_argument("--method", default="fused", choices=["fused", "sweep"])
    ap.add_argument("--mapping", default="cell", choices=["cell", "sa"])
    ap.add_argument("--dtype", default="f32", choices=["f32", "f64"])
    ap.add_argument("--gamma", type=float, default=0.99)
    ap.add_argument("--tol", type=float, default=1e-6)
    ap.add_argument("--cpu-budget", type=float, default=8.0, help="seconds of CPU baseline sampling")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-hbm", action="store_true", help="skip the HBM-roofline side measurement")
    ap.add_argument("--no-f64", action="store_true", help="skip the fp64 (parity-mode) side measurement")
    ap.add_argument("--no-sharded", action="store_true", help="skip the sharded lava65536 / doorkey65536 blocks")
    args = ap.parse_args()

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    if os.environ.get("MGDP_BENCH_DRYRUN") == "1":
        return dry_run(args, rank, world)
    # Rehearsal knobs for a 1-GPU box (never set by the driver): MGDP_BENCH_DEVICE pins every rank
    # to one device, MGDP_BENCH_BACKEND=gloo replaces RCCL (which refuses two ranks per GPU).
    local = int(os.environ.get("MGDP_BENCH_DEVICE", local))
    backend = os.environ.get("MGDP_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local)
    # The solving (main) thread on the CPUs of its GPU's NUMA node, before any handle exists (its
    # host-mapped words are allocated by this thread): a served lone-grid solve measured 9.1 us from
    # the GPU's node and 10.8 us from the other socket (tools/probe_numa.cpp).
    # MGDP_BENCH_PIN=0 leaves the thread where the scheduler put it.
    from minigrid_dynamicprogramming_amd import _lib as mglib

    pinned = mglib.pin_host_thread(local) if os.environ.get("MGDP_BENCH_PIN", "1") == "1" else 0
    # MGDP_BENCH_FORCE_DIST=1 (rehearsal, never set by the driver): the process group and the sharded
    # protocol at any world size, so one GPU runs the RCCL all-reduces of the multi-GPU path
    force_dist = os.environ.get("MGDP_BENCH_FORCE_DIST") == "1"
    dist = None
    if world > 1 or force_dist:
        import torch.distributed as dist

        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    red_dev = torch.device("cuda", local) if backend == "nccl" else torch.device("cpu")

    if args.workload in STEP_WORKLOADS or args.workload in GEN_WORKLOADS:
        side = step_bench if args.workload in STEP_WORKLOADS else gen_bench
        out = side(args, rank, world, local, dist, red_dev)
        if rank == 0:
            print(json.dumps(out), flush=True)
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    reducer_box = []

    def get_reducer():
        # the library's own communicator (mgdp_vi_solve_sharded: RCCL called from libmgdp, one C call
        # per solve) under RCCL; MGDP_BENCH_LIB_COMM=0 keeps the torch.distributed protocol
        if not reducer_box and backend == "nccl" and os.environ.get("MGDP_BENCH_LIB_COMM", "1") != "0":
            from minigrid_dynamicprogramming_amd.distributed import LibComm

            # every rank takes the library's communicator or none does.  The ranks first agree on a
            # LOCAL check (librccl loads: mgdp_comm_available), with one MIN all-reduce, and only then
            # start the collective bootstrap (the id broadcast and ncclCommInitRank): a rank that
            # cannot load librccl sends the whole job to the torch.distributed protocol before any
            # rank waits in a collective the others never join.  A failure inside ncclCommInitRank
            # itself (after agreement) leaves its peers waiting there and cannot be recovered from.
            err = ""
            try:
                if os.environ.get("MGDP_BENCH_LIB_COMM_FAIL") == str(rank):  # rehearsal of the fallback
                    raise RuntimeError("MGDP_BENCH_LIB_COMM_FAIL")
                here = LibComm.available()
                if not here:
                    err = "librccl could not be loaded"
            except Exception as ex:  # noqa: BLE001 -- reported, then the torch path
                here, err = False, f"{type(ex).__name__}: {ex}"
            ok = torch.tensor([1 if here else 0], dtype=torch.int32, device=red_dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            if int(ok.item()) == 1:
                reducer_box.append(LibComm(device=local))
            else:
                log(f"[rank {rank}] library communicator unavailable ({err or 'unavailable on another rank'}); "
                    "torch.distributed protocol instead")
        if not reducer_box:
            from minigrid_dynamicprogramming_amd.distributed import Reducer

            reducer_box.append(Reducer(timing=True))  # built once; its stream carries the shards' launches
        return reducer_box[0]

    def run_workload(name, dtype=None, split_events=False):
        spec = WORKLOADS[name]
        t_gen = time.perf_counter()
        cells, (lo, hi) = make_cells(spec, rank, world)
        log(f"[rank {rank}] {name}: grids [{lo},{hi}) generated in {time.perf_counter() - t_gen:.1f}s")
        sharded = spec["sharded"] and (world > 1 or force_dist)
        wargs = argparse.Namespace(**{**vars(args), "workload": name})
        fresh = None
        if split_events and not spec.get("replicate") and not spec.get("distinct") and FRESH_SETS > 0:
            # fresh grid sets for the first-solve timing: seeds shifted past the workload's own
            n_all = spec["global_grids"] if spec["sharded"] else spec["per_gpu"] * world
            fresh = [make_cells(spec, rank, world, seed_offset=(i + 1) * n_all)[0] for i in range(FRESH_SETS)]
        m = measure(wargs, dtype or args.dtype, cells, local, dist, red_dev, get_reducer() if sharded else None, sharded,
                    split_events=split_events, fresh=fresh)
        return spec, cells, (lo, hi), sharded, m

    # the BASELINE configs 3-5 beside the default line (every rank takes part), run BEFORE the
    # headline: on a fresh box the device and host clocks are then at their working state when the
    # lone-grid server starts (the driver measured 11.3 us per solve first-in-process vs 9.3 us for
    # the fp64 line after these blocks, round 3); the headline's priming rule still applies
    blocks, batched = {}, {}
    if args.workload == "empty16" and not args.no_sharded and args.method == "fused" and args.mapping == "cell":
        # BASELINE configs 3-5 beside the headline: FourRooms x 4096 per GPU (independent batches),
        # LavaS11N5 / DoorKey-16 x 65536 sharded over the N ranks; each with the oracle timed on a
        # bounded sample of the same grids at N = 1
        for name in ("fourrooms4096", "lava65536", "doorkey65536"):
            bspec, bcells, (blo, bhi), bsharded, bm = run_workload(name, split_events=True)
            if rank == 0:
                blk = {"value": bm["upd_total"] / bm["elapsed_max"], "unit": "updates/s",
                       "ms_per_solve": bm["elapsed_max"] * 1000.0 / args.steps, "sweeps": int(bm["sweeps"][-1]),
                       "env_id": bspec["env_id"], "grids_rank0": bhi - blo, "dtype": args.dtype}
                if bspec["sharded"]:
                    blk.update({"global_grids": bspec["global_grids"], "scaling": "strong",
                                "parallelism": (f"shard{world} + RCCL all-reduce" if bsharded and backend == "nccl" else
                                                f"shard{world} + {backend} all-reduce" if bsharded else "direct (one GPU)")})
                else:
                    blk.update({"global_grids": (bhi - blo) * world, "scaling": "weak",
                                "parallelism": f"independent batches x{world}"})
                blk["roofline"] = workload_roofline(args, args.dtype, bm, name, bhi - blo)
                if not bm["events_in_region"]:
                    blk["roofline"]["events"] = ("launch durations from a second pass of the same solves with "
                                                 "per-launch HIP events (they cost 6-9 us of host time per "
                                                 "launch, so the timed region runs without them)")
                if bm.get("executed"):
                    blk["executed_rank0"] = bm["executed"]
                    blk["executed_updates_per_s"] = blk["value"] * bm["executed"]["frac_of_global_rule"]
                if bm.get("collectives"):
                    blk["collectives"] = bm["collectives"]
                if bm.get("fresh"):
                    blk["fresh"] = bm["fresh"]
                if world == 1 and not args.no_cpu:
                    model = bm["info"]["model"]
                    blk["cpu_baseline"] = cpu_baseline(bcells, model, args.gamma, args.tol, args.dtype, BLOCK_CPU_S)
                    blk["cpu_baseline_all_cores"] = cpu_baseline(bcells, model, args.gamma, args.tol, args.dtype,
                                                                 BLOCK_CPU_S, nthreads=host_cores())
                    # like-for-like: the oracle with the same per-grid fixed-point stop as the GPU
                    blk["cpu_baseline_fp"] = cpu_baseline(bcells, model, args.gamma, args.tol, args.dtype,
                                                          BLOCK_CPU_S, fixed_point=True)
                    blk["cpu_baseline_fp_all_cores"] = cpu_baseline(bcells, model, args.gamma, args.tol, args.dtype,
                                                                    BLOCK_CPU_S, nthreads=host_cores(),
                                                                    fixed_point=True)
                (blocks if bspec["sharded"] else batched)[name] = blk
    # MGDP_BENCH_SPLIT_EVENTS=1 (rehearsal knob, tools/gpu_shard_prof.sh): the main line's region
    # without per-launch events too, as the blocks beside the headline run it
    spec, cells, (lo, hi), sharded, m = run_workload(args.workload,
                                                     split_events=os.environ.get("MGDP_BENCH_SPLIT_EVENTS") == "1")
    if rank != 0:  # the fp64 side line and the CPU baselines are N = 1 only
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return
    vi_info = m["info"]
    roofline = workload_roofline(args, args.dtype, m, args.workload, hi - lo)
    out = {
        "metric": METRIC,
        "value": m["upd_total"] / m["elapsed_max"],
        "unit": "updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": m["elapsed_max"] * 1000.0 / args.steps,
        "higher_is_better": True,
        "scaling": "strong" if spec["sharded"] else "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": f"synthetic: {spec['env_id']} grids from the reference-exact generator "
                f"({'seed 0 replicated' if spec['replicate'] else 'seeds ' + str(lo) + '..'})",
        "config": {
            "workload": args.workload, "env_id": spec["env_id"], "grids_per_gpu": hi - lo,
            "global_grids": (hi - lo) * world if not spec["sharded"] else spec["global_grids"],
            "states_per_grid": vi_info["S"], "actions": vi_info["A"], "gamma": args.gamma, "tol": args.tol,
            "method": args.method, "mapping": args.mapping,
            "parallelism": (f"shard{world} + RCCL dV all-reduce" if sharded else
                            ("replicas only" if spec["replicate"] else f"independent batches x{world}")),
            "host_thread": (f"pinned to the GPU's NUMA node ({pinned} CPUs)" if pinned else "unpinned"),
            **({"emulated_shard_of": shard_of(world)} if spec["sharded"] and shard_of(world) != world else {}),
        },
        "sweeps": int(m["sweeps"][-1]),
        "roofline": roofline,
        **({"sweeps_mean": float(np.mean(m["sweeps"])), "distinct_grids": len(cells)} if spec.get("distinct") else {}),
    }
    if m.get("collectives"):
        out["collectives"] = m["collectives"]
    if m.get("latency"):
        out["latency"] = m["latency"]
    if m.get("executed"):
        out["executed_rank0"] = m["executed"]
    if batched:
        out["batched"] = batched
    if blocks:
        out["sharded"] = blocks
    if args.dtype == "f32" and world == 1 and not args.no_f64:
        m64 = measure(args, "f64", cells, local, dist, red_dev, get_reducer() if sharded else None, sharded)
        out["f64"] = {"value": m64["upd_total"] / m64["elapsed_max"], "unit": "updates/s",
                      "ms_per_step": m64["elapsed_max"] * 1000.0 / args.steps, "sweeps": int(m64["sweeps"][-1]),
                      "kernel": m64["info"]["kernel"],
                      "note": "same workload and steps in fp64 (parity mode: bit-exact with the fp64 oracle)"}

    if world == 1 and not args.no_hbm and args.workload == "empty16":
        out["roofline_hbm"] = hbm_side_measurement(args)
    if world == 1 and not args.no_cpu:
        out["host"] = host_info()
        lone = bool(spec.get("distinct"))
        out["cpu_baseline"] = cpu_baseline(cells, vi_info["model"], args.gamma, args.tol, args.dtype, args.cpu_budget,
                                           lone=lone)
        out["cpu_baseline_all_cores"] = cpu_baseline(
            cells, vi_info["model"], args.gamma, args.tol, args.dtype, max(2.0, args.cpu_budget / 4),
            nthreads=out["host"]["cores_used"], lone=lone)
        out["cpu_baseline_numpy"] = numpy_baseline(cells, vi_info["model"], args.gamma, args.tol, args.dtype,
                                                   max(2.0, args.cpu_budget / 4))
    emit(out)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def _g(x, n=4):
    """x rounded to n significant digits (None passes)."""
    return None if x is None else float(f"{x:.{n}g}")


def compact_line(out: dict) -> dict:
    """The stdout line: the contract's keys, a short roofline and CPU leg, and one summary per BASELINE
    config measured beside the headline -- small enough (< 2000 chars) that a driver keeping only the
    tail of stdout still holds all of it.  The full record goes to stderr / MGDP_BENCH_DETAIL."""
    c = {k: out[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                             "higher_is_better", "scaling", "vs_baseline", "dtype") if k in out}
    c["value"], c["ms_per_step"] = _g(out["value"], 6), _g(out["ms_per_step"], 5)
    c["data"] = out["data"].split(" grids from")[0] + " grids, reference-exact generator"
    cfg = out["config"]
    c["config"] = {k: cfg[k] for k in ("workload", "env_id", "grids_per_gpu", "global_grids", "states_per_grid",
                                       "actions", "gamma", "tol", "method", "parallelism") if k in cfg}
    c["sweeps"] = out.get("sweeps")
    r = out["roofline"]
    c["roofline"] = {"bound": r["bound"], "kernel": r["kernel"], "achieved": _g(r["achieved"]), "peak": r["peak"],
                     "unit": r["unit"], "frac": _g(r["frac"], 3), "traffic": _g(r.get("traffic")),
                     "avg_launch_us": _g(r.get("avg_launch_us"), 5), "launches": r.get("launches"),
                     "solves_per_launch": r.get("solves_per_launch")}
    cb = out.get("cpu_baseline")
    if cb:
        c["cpu_baseline"] = {"value": _g(cb["value"]), "unit": cb["unit"], "cores": cb["cores"], "kind": cb["kind"],
                             "sample": cb["sample"].split(" of the same workload")[0] + ", oracle C"}
    if out.get("collectives"):
        col = out["collectives"]
        c["collectives"] = {k: col[k] for k in ("allreduces_per_solve", "host_reads_per_solve") if k in col}
        c["collectives"]["path"] = "libmgdp" if "libmgdp" in col.get("path", "") else "torch"
    lat = out.get("latency") or {}
    if lat.get("gpu_solve_us") is not None:
        c["lat_us"] = {"gpu": lat["gpu_solve_us"], "host": lat.get("host_and_handoff_us")}
    cfgs = {}
    if out.get("cpu_baseline_all_cores"):
        cfgs[cfg["workload"]] = {"v": _g(out["value"]), "ms": _g(out["ms_per_step"]), "k": out.get("sweeps"),
                                 "c1": _g(cb["value"]) if cb else None, "c16": _g(out["cpu_baseline_all_cores"]["value"])}
    for grp in ("batched", "sharded"):
        for name, b in (out.get(grp) or {}).items():
            e = b.get("executed_rank0") or {}
            v = (b.get("roofline") or {}).get("valu") or {}
            d = {"v": _g(b["value"]), "x": _g(b.get("executed_updates_per_s")), "ms": _g(b["ms_per_solve"]),
                 "msf": _g((b.get("fresh") or {}).get("ms_per_solve")), "msa": _g((b.get("fresh") or {}).get("ms_per_solve_again")),
                 "kf": _g((b.get("fresh") or {}).get("kernel_ratio"), 3),
                 "k": b["sweeps"], "xf": _g(e.get("frac_of_global_rule"), 3), "valu": _g(v.get("frac"), 2)}
            for key, src in (("c1", "cpu_baseline"), ("c16", "cpu_baseline_all_cores"), ("f1", "cpu_baseline_fp"),
                             ("f16", "cpu_baseline_fp_all_cores")):
                if b.get(src):
                    d[key] = _g(b[src]["value"])
            cfgs[name] = {k: x for k, x in d.items() if x is not None}
    if cfgs:
        c["configs"] = cfgs
        c["configs_keys"] = ("v upd/s as the metric counts (B*S*A*K); x executed upd/s; ms per solve; msf/msa ms of "
                             "the 1st/2nd solve of fresh grids (1-solve regions), kf their kernel ratio; k sweeps; "
                             "xf executed/K; valu VALU frac; c1/c16 CPU oracle 1/16 threads; f1/f16 same, per-grid "
                             "fixed-point stop")
    return c


def emit(out: dict):
    """Full record to stderr (and MGDP_BENCH_DETAIL=path), then the compact line on stdout, last."""
    detail = json.dumps(out)
    log("bench detail: " + detail)
    path = os.environ.get("MGDP_BENCH_DETAIL")
    if path:
        with open(path, "w") as f:
            f.write(detail + "\n")
    print(compact_dumps(compact_line(out)), flush=True)


def compact_dumps(obj) -> str:
    """json.dumps without spaces, large numbers in exponent form (the values are already rounded to
    <= 6 significant digits): 24443600000.0 -> 2.44436e+10."""
    import re

    txt = json.dumps(obj, separators=(",", ":"))
    return re.sub(r'(?<=[:\[,])(\d{7,}(?:\.\d+)?)(?=[,}\]])', lambda m: f"{float(m.group(1)):.6g}", txt)


def compulsory_bytes_per_solve(info, tsize, method, sweeps):
    """Bytes a solve must move between HBM and the CUs.  fused / served: the grid's cells in, V and
    pi out, once per solve (V stays in LDS across sweeps); sweep: SURVEY 8(d)'s 2*S*sizeof V + W*H
    per grid-sweep (V read and written every sweep) plus the pi pass."""
    B, S, HW = info["B"], info["S"], info["W"] * info["H"]
    if method == "fused":
        return B * (HW + S * tsize + S)
    return B * (compulsory_bytes_per_sweep(S, HW, tsize) * sweeps + S * tsize + HW + S)


def measure(args, dtype, cells, local, dist, red_dev, reducer, sharded, split_events=False, fresh=None):
    """W warmup solves, then K timed solves (barrier + synchronize on both sides, max over ranks).
    split_events (the BASELINE-config blocks beside the headline): the timed region runs without the
    library's per-launch HIP events -- on a batched solve they cost 6-9 us of host time per launch
    (tools/probe_timing_cost.py, profiles/r04_tcost/) -- and the launch durations for the roofline
    come from a second pass of the same K solves with the events on."""
    import torch

    import minigrid_dynamicprogramming_amd as mg
    from minigrid_dynamicprogramming_amd.distributed import solve_sharded

    distinct = WORKLOADS[args.workload].get("distinct")
    vi = mg.ValueIteration(cells[:1] if distinct else cells, gamma=args.gamma, tol=args.tol, dtype=dtype,
                           method=args.method, mapping=args.mapping, device=local)
    if distinct:
        # the grids stay resident in HBM; step i hands grid i mod n to the solver (device pointer)
        grids = torch.from_numpy(np.ascontiguousarray(cells)).to(f"cuda:{local}")
        torch.cuda.synchronize()
        base, hw, n_grids = grids.data_ptr(), cells.shape[1] * cells.shape[2], len(cells)
        nxt = [0]

    def one_solve(last=False):
        if sharded:
            if type(reducer).__name__ == "LibComm":
                return solve_sharded(vi, comm=reducer)["sweeps"]
            return solve_sharded(vi, reducer=reducer)["sweeps"]
        if distinct:
            vi.load_device(base + (nxt[0] % n_grids) * hw)
            nxt[0] += 1
        return vi.solve(last)

    def barrier():
        if dist is not None:
            dist.barrier()

    # Warmup runs the timed sequence itself, edges included: timing on, W solves, then the same
    # end-of-region teardown (a resident lone-grid server leaves, stream and device drained), so
    # no first-time cost of that path lands in the timed region.
    split = split_events and not vi.persistent
    vi.enable_timing(not split)
    wstamps = [time.perf_counter()]
    for i in range(args.warmup):
        one_solve(last=i == args.warmup - 1)
        wstamps.append(time.perf_counter())
    if split and not sharded:
        # the BASELINE-config blocks: the W warmup solves of a batch last well under a millisecond, so the
        # device's clock has not ramped when the region starts; keep solving for PRIME_BLOCK_S first (the
        # headline's priming rule, shorter: a batched solve does far more work per call)
        while time.perf_counter() - wstamps[0] < PRIME_BLOCK_S:
            one_solve()
    vi.synchronize()
    torch.cuda.synchronize()
    warm_us = [(b - a) * 1e6 for a, b in zip(wstamps[:-1], wstamps[1:])]
    # Re-enabling timing drops the warmup's launches; a persistent handle then gets untimed
    # priming solves, which relaunch the server (its launch is timed from here), so the timed
    # region holds no relaunch and its length does not depend on --steps.
    vi.enable_timing(not split)
    if reducer is not None:
        reducer.collect()
        reducer.reset_counters()
        reducer.timing = reducer.device.type == "cuda" and not split  # its events too: the events pass
    barrier()
    torch.cuda.synchronize()
    # Priming to a steady state (persistent lone-grid server), in two phases.
    # (1) warm: solves for at least PRIME_MIN_S, then windows of PRIME_WIN solves until a window's
    #     median latency is within PRIME_TOL of the previous window's (at most PRIME_MAX_S in all):
    #     a device or host core that was idle ramps its clock over milliseconds (the driver's fresh
    #     box, round 3: 11.3 us per solve after 16 priming solves; warm boxes 7.9-8.8 us).  That
    #     server then leaves: a launch that lived ~0.2 s closes slowly and erratically (the stream's
    #     completion 9-65 us after its exit word vs 6-8 us for a young one, tools/probe_edge.py,
    #     profiles/r04_edge/), which would land in the region's closing edge.
    # (2) relaunch: PRIME_RELAUNCH solves on a new server launch (the first solves after a relaunch
    #     run 3-4 us slower), timed from here, the last one right before the region -- the first
    #     timed solve must find the server busy-polling (the solve fast path wants the last request
    #     < 50 us old; past that it takes the general path and may relaunch).
    primed = 0
    pstamps = [time.perf_counter()]
    prime_meds = []
    warm_clock = None
    if vi.persistent:
        t_prime = pstamps[0]
        while time.perf_counter() - t_prime < PRIME_MAX_S:
            for _ in range(PRIME_WIN):
                one_solve()
                primed += 1
                pstamps.append(time.perf_counter())
            if pstamps[-1] - t_prime < PRIME_MIN_S:
                continue
            w = np.diff(pstamps[-PRIME_WIN - 1:]) * 1e6
            prime_meds.append(float(np.median(w)))
            if len(prime_meds) >= 2 and abs(prime_meds[-1] - prime_meds[-2]) <= PRIME_TOL * prime_meds[-2]:
                break
        one_solve(last=True)
        primed += 1
        vi.synchronize()
        warm_clock = vi.serve_clock()
        vi.enable_timing(True)  # the timed launch is the relaunch below
        torch.cuda.synchronize()
        pstamps.append(time.perf_counter())
        for _ in range(PRIME_RELAUNCH):
            one_solve()
            primed += 1
            pstamps.append(time.perf_counter())
    if split and not sharded:
        # a resident batch server (vi_bserve_kernel, round 6) left at the timing switch and the device
        # synchronize above: one more untimed solve relaunches it right before the region (as the lone
        # server's relaunch priming does), so the region times served solves, not a relaunch per K
        one_solve()
    stamps = [] if os.environ.get("MGDP_BENCH_STAMPS") else None  # diagnostics: where the region's time goes
    # the plain case calls the bound solve() directly (no wrapper, no per-step argument): a served
    # lone grid answers in a few microseconds and the loop's own Python is part of each step's host turnaround
    lean = not sharded and not distinct and stamps is None
    solve = vi.solve
    t0 = time.perf_counter()
    sweeps = []
    if lean:
        for _ in range(args.steps - 1):
            sweeps.append(solve())
        sweeps.append(solve(True))
    for i in range(0 if lean else args.steps):
        # the last solve dismisses a resident lone-grid server (mgdp_vi_solve_last) instead of the
        # synchronize below telling it to leave
        sweeps.append(one_solve(last=i == args.steps - 1))
        if stamps is not None:
            stamps.append(time.perf_counter())
    # make the last solve final: a resident lone-grid server is told to leave (it exits within a
    # poll) and the stream drained; a device synchronize alone would wait out the server's idle limit
    vi.synchronize()
    if stamps is not None:
        stamps.append(time.perf_counter())
    torch.cuda.synchronize()
    if stamps is not None:
        stamps.append(time.perf_counter())
    # Each rank's region ends at its own completion and the job's time is the max over ranks (the
    # all-reduce below); the closing barrier only re-aligns the ranks, and its own latency (a
    # gloo / RCCL barrier measured 150-200 us, 8-9 us per solve over 20 solves,
    # profiles/r02_dist_penalty/) is not work, so it stays outside the region.
    elapsed = time.perf_counter() - t0
    barrier()
    if stamps is not None:
        us = [(b - a) * 1e6 for a, b in zip([t0] + stamps[:-1], stamps)]
        pr_us = [round((b - a) * 1e6, 2) for a, b in zip(pstamps[:-1], pstamps[1:])]
        log(json.dumps({"stamps_us": {"prime_n": len(pr_us), "prime_first16": pr_us[:16], "prime_last16": pr_us[-16:],
                                      "gap": round((t0 - pstamps[-1]) * 1e6, 2),
                                      "solves": [round(x, 2) for x in us[:-2]], "vi_sync": round(us[-2], 2),
                                      "dev_sync": round(us[-1], 2), "region": round(elapsed * 1e6, 2)}}))
    red_region = None
    if reducer is not None:  # the region's protocol counters (the events pass below adds its own)
        red_region = (reducer.calls, reducer.host_reads, reducer.wall_s)
    if split:  # the roofline's launch durations: the same K solves again, per-launch events on
        vi.enable_timing(True)
        if reducer is not None:
            reducer.reset_counters()
            reducer.timing = reducer.device.type == "cuda"
        for i in range(args.steps):
            one_solve()
        vi.synchronize()
    kern_ms, launches = vi.kernel_time()
    clock = vi.serve_clock() if vi.persistent else None
    gsw = vi.grid_sweeps() if vi.B > 1 else None  # sweeps each grid executed in the last solve
    vi.enable_timing(False)
    fresh_out = None
    if fresh:
        # First solves of FRESH grids (round 6): a new grid set is loaded -- uploaded,
        # its dispatch order computed from the cells -- outside the timing, then ONE solve is timed like
        # a region of one step (the solve and the closing synchronize), on every rank at once; the max
        # over ranks of each, then the median over the sets.  The repeated region above solves the same
        # grids K times; this says what a user solving new grids every time gets.
        def one_timed():
            barrier()
            torch.cuda.synchronize()
            vi.enable_timing(True)
            t = time.perf_counter()
            k_f = one_solve()
            vi.synchronize()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            kms, _ = vi.kernel_time()
            vi.enable_timing(False)
            if dist is not None:
                tt = torch.tensor([dt, kms], dtype=torch.float64, device=red_dev)
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                dt, kms = float(tt[0].item()), float(tt[1].item())
            return dt, kms, k_f

        first, again = [], []
        for fc in fresh:
            vi.load(fc)
            first.append(one_timed())  # the first solve of these grids
            again.append(one_timed())  # the same grids once more, timed the same way (one solve + its edge)
        med = lambda xs, i: round(float(np.median([x[i] for x in xs])) * (1e3 if i == 0 else 1.0), 5)
        fresh_out = {"ms_per_solve": med(first, 0), "ms_per_solve_again": med(again, 0),
                     "kernel_ms": med(first, 1), "kernel_ms_again": med(again, 1),
                     "ratio": round(med(first, 0) / med(again, 0), 4),
                     "kernel_ratio": round(med(first, 1) / med(again, 1), 4), "sets": len(first),
                     "ms_each": [round(x[0] * 1e3, 5) for x in first], "sweeps": [x[2] for x in first],
                     "rule": "per set: load (upload + dispatch order from the cells, untimed), then ONE timed solve "
                             "+ the closing synchronize (a region of one step, so its edge is not amortized as in "
                             "the K-step region; per-launch events on), then the same grids once more, timed the "
                             "same way; max over ranks, median over sets.  kernel_ms: the launches' event time"}
    info = {"A": 7 if vi.model == "xyd" else 5, "W": vi.W, "H": vi.H, "S": vi.S, "B": vi.B, "model": vi.model,
            "updates_per_sweep": vi.updates_per_sweep, "kernel": vi.kernel_name, "persistent": vi.persistent}
    vi.close()
    upd_rank = float(info["updates_per_sweep"]) * float(sum(sweeps))
    collectives = None
    if reducer is not None:
        dev_ms = reducer.collect()
        calls, reads, wall_s = red_region
        if type(reducer).__name__ == "LibComm":
            collectives = {"allreduces_per_solve": calls / args.steps, "host_reads_per_solve": reads / args.steps,
                           "path": "libmgdp communicator (mgdp_vi_solve_sharded: RCCL enqueued by the library on "
                                   "the handle's stream, one C call per solve; host waits counted by the library, "
                                   "mgdp_comm_host_waits)"}
        else:
            collectives = {"allreduces_per_solve": calls / args.steps,
                           "host_reads_per_solve": reads / args.steps,
                           "allreduce_us_per_solve_rank0": dev_ms * 1000.0 / args.steps,
                           "protocol_host_us_per_solve_rank0": wall_s * 1e6 / args.steps,
                           "path": f"torch.distributed {dist.get_backend() if dist is not None else '-'} "
                                   "process group (distributed.Reducer)",
                           "note": "device time of the all-reduces (events on the protocol stream, includes "
                                   "waiting for the slowest rank; from the events pass when the region runs "
                                   "without events; 0 on a CPU-side gloo group) and host time of the one read "
                                   "per solve"}
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        u = torch.tensor([upd_rank], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(u, op=dist.ReduceOp.SUM)
        elapsed_max, upd_total = float(t.item()), float(u.item())
    else:
        elapsed_max, upd_total = elapsed, upd_rank
    lat = None
    if info["persistent"] or distinct:
        pr = np.diff(pstamps) * 1e6
        lat = {"first_solve_us": round(warm_us[0], 2) if warm_us else None,
               "warmup_solves_us": [round(x, 2) for x in warm_us],
               "priming_solves": primed, "priming_ms": round(float(pr.sum()) / 1e3, 2) if len(pr) else 0.0,
               "priming_first16_us": [round(x, 2) for x in pr[:16]],
               "priming_window_medians_us": [round(x, 3) for x in prime_meds],
               "priming_last_window_median_us": prime_meds[-1] if prime_meds else None,
               "steady_rule": f"solves for >= {PRIME_MIN_S * 1e3:.0f} ms, then windows of {PRIME_WIN} solves "
                              f"until a window's median is within {PRIME_TOL:.0%} of the previous "
                              f"(at most {PRIME_MAX_S * 1e3:.0f} ms); that server leaves, then "
                              f"{PRIME_RELAUNCH} solves on the relaunched (timed) server before the region"}
        if warm_clock and warm_clock["launches"]:
            lat["warm_phase_clock"] = warm_clock
        if clock and clock["launches"]:
            lat["device_clock"] = {**clock, "source": "vi_serve_kernel s_memtime cycles / s_memrealtime over the "
                                                      "timed launch (relaunch priming + timed solves)"}
            if clock.get("gpu_solve_us"):
                # where a solve's time goes: on the GPU (request seen -> solve end) vs the rest
                # (host call, request / result over PCIe, the region's edges)
                lat["gpu_solve_us"] = round(clock["gpu_solve_us"], 3)
                lat["host_and_handoff_us"] = round(elapsed * 1e6 / args.steps - clock["gpu_solve_us"], 3)
    executed = None
    if gsw is not None and sweeps[-1] > 0:
        executed = {"mean_grid_sweeps": round(float(gsw.mean()), 3), "global_sweeps": int(sweeps[-1]),
                    "frac_of_global_rule": round(float(gsw.mean()) / sweeps[-1], 4),
                    "note": "fixed-point completion: a grid whose own rule stopped at an exact fixed point "
                            "(|dV| = 0) is complete for the global K (V, pi bit-identical), its remaining "
                            "K - k_e sweeps are not executed; value counts B*S*A*K as the metric defines"}
    return {"elapsed_max": elapsed_max, "upd_total": upd_total, "sweeps": sweeps, "kern_ms": kern_ms,
            "events_in_region": not split,
            "executed": executed,
            "launches": launches, "primed": primed, "timed_primed": PRIME_RELAUNCH if info["persistent"] else 0,
            "info": info, "collectives": collectives, "latency": lat, "fresh": fresh_out}


def host_cores() -> int:
    """CPU threads the baseline may use: the affinity set, capped by OMP_NUM_THREADS (the pool's
    per-GPU CPU share on the box)."""
    aff = len(os.sched_getaffinity(0))
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        return max(1, min(aff, int(os.environ["OMP_NUM_THREADS"])))
    return aff


def host_info():
    """The CPU the baseline runs on: nproc / affinity (the whole machine on the GPU box) and the
    cores this process is allotted (OMP_NUM_THREADS: the pool's per-GPU CPU share), lscpu model."""
    import subprocess

    aff = len(os.sched_getaffinity(0))
    cores = host_cores()
    model = ""
    try:
        for line in subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout.splitlines():
            if line.startswith("Model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    nproc = os.cpu_count()
    try:
        nproc = int(subprocess.run(["nproc"], capture_output=True, text=True, timeout=10).stdout.strip())
    except Exception:
        pass
    from minigrid_dynamicprogramming_amd import _lib

    return {"nproc": nproc, "affinity_cpus": aff, "cores_used": cores, "cpu_model": model,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "hip_runtime": _lib.hip_runtime()}  # which libamdhip64 serves libmgdp (torch's when imported first)


def numpy_baseline(cells, model, gamma, tol, dtype, budget_s):
    """oracle/numpy_vi.py (numpy Jacobi restatement, single thread) on the same sample."""
    from oracle.numpy_vi import NumpyVI

    # 32 grids per thread (a threaded batch solve needs work for every thread), 32 for one thread
    sample = cells[: min(len(cells), 32)]
    n = NumpyVI(0 if model == "xyd" else 1, sample, gamma, tol, dtype)
    solves, upd, k = 0, 0, 0
    t0 = time.perf_counter()
    while True:
        r = n.solve()
        k = r["sweeps"]
        upd += n.B * n.S * n.A * k
        solves += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    el = time.perf_counter() - t0
    return {"value": upd / el, "unit": "updates/s", "cores": 1, "kind": "port",
            "sample": f"{solves} full solves of {n.B} grid(s) ({k} sweeps each, {dtype}), oracle/numpy_vi.py "
                      f"(vectorised numpy Jacobi over the oracle's transition tables), {el:.1f} s"}


def _max_over_ranks(dist, red_dev, elapsed, units):
    import torch

    if dist is None:
        return elapsed, units
    t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
    u = torch.tensor([units], dtype=torch.float64, device=red_dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(u, op=dist.ReduceOp.SUM)
    return float(t.item()), float(u.item())


def _timed_launches(args, launch, dist, stream=None):
    """W untimed launches, then K launches bracketed by barrier + synchronize, each launch between
    a pair of events on `stream`, the stream the library launches on (a torch Stream; None = the
    current stream).  The events must be on the launch stream: events on another stream time
    nothing (round-1 lesson: the legacy null stream handle 0 made the library create its own)."""
    import torch

    if stream is not None:
        with torch.cuda.stream(stream):
            return _timed_launches(args, launch, dist)
    for i in range(args.warmup):
        launch(i)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        evs[i][0].record()
        launch(args.warmup + i)
        evs[i][1].record()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0  # before the closing barrier (see measure())
    if dist is not None:
        dist.barrier()
    kern_s = sum(a.elapsed_time(b) for a, b in evs) / 1000.0
    return elapsed, kern_s


def step_bench(args, rank, world, local, dist, red_dev):
    """K batched steps (MiniGridEnv.step + gen_obs, one envs_step_kernel launch
    each) of B envs resident in HBM, actions pre-drawn on the device; env-steps/s."""
    import torch

    from minigrid_dynamicprogramming_amd.vector import MiniGridVecEnv

    spec = STEP_WORKLOADS[args.workload]
    B = spec["per_gpu"]
    venv = MiniGridVecEnv(spec["env_id"], B, device=local)
    venv.reset(seed=rank * B)  # reset(seed) for seeds [rank*B, (rank+1)*B), generated on the GPU
    dev = torch.device("cuda", local)
    stream = torch.cuda.Stream(device=dev)  # a real stream handle (0 would make the library use its own)
    venv.set_stream(stream.cuda_stream)
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    acts = torch.randint(0, 7, (args.warmup + args.steps, B), generator=g, device=dev, dtype=torch.int32)
    V = venv.view
    obs = torch.empty((B, V, V, 3), dtype=torch.uint8, device=dev)
    dirn = torch.empty(B, dtype=torch.int32, device=dev)
    rew = torch.empty(B, dtype=torch.float64, device=dev)
    term = torch.empty(B, dtype=torch.uint8, device=dev)
    trunc = torch.empty(B, dtype=torch.uint8, device=dev)
    status = torch.empty(B, dtype=torch.int32, device=dev)

    # raw device pointers: the per-launch host cost is the ctypes call alone
    act_ptrs = [acts[i].data_ptr() for i in range(acts.shape[0])]
    outs = tuple(t.data_ptr() for t in (obs, dirn, rew, term, trunc, status))

    def launch(i):
        venv.step_device(act_ptrs[i], *outs)

    torch.cuda.synchronize()  # actions / outputs allocated on the default stream
    # Kernel time: one HIP event pair on the launch stream around the K back-to-back launches.  The
    # host issues a launch in less time than the kernel runs (tools/probe_step: 2.7 us per call vs
    # 11 us), so the stream stays busy and (end - start) / K is the launch duration plus the
    # inter-dispatch gap -- a conservative per-launch time.  Per-launch event pairs
    # (mgdp_envs_enable_timing) cost ~8 us of host time per launch and would throttle the loop.
    for i in range(args.warmup):
        launch(i)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        launch(args.warmup + i)
    ev1.record(stream)
    stream.synchronize()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0  # before the closing barrier (see measure())
    if dist is not None:
        dist.barrier()
    kern_s = ev0.elapsed_time(ev1) / 1000.0
    assert int(status.max().item()) == 0, "step kernel reported an error status"
    elapsed_max, steps_total = _max_over_ranks(dist, red_dev, elapsed, float(B) * args.steps)
    out = None
    if rank == 0:
        bpe = step_bytes_per_env_step(V)
        avg = kern_s / args.steps
        ach = bpe * B / avg / 1e9
        out = {
            "metric": "batched env steps/sec (MiniGridEnv.step + gen_obs), " + spec["env_id"],
            "value": steps_total / elapsed_max, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed_max * 1000.0 / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": f"synthetic: {spec['env_id']} reset(seed) grids for seeds [{rank * B}, ..) generated on the "
                    "GPU, uniform random actions 0..6 drawn on the device (no resets inside the timed region)",
            "config": {"workload": args.workload, "env_id": spec["env_id"], "envs_per_gpu": B,
                       "global_envs": B * world, "view": V, "parallelism": f"independent env batches x{world}"},
            "roofline": {"bound": "hbm", "kernel": "envs_step_kernel", "achieved": ach, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                         "traffic": load_traffic(f"{args.workload}/step", 1.0, grids=B), "launches": args.steps,
                         "avg_launch_us": avg * 1e6, "alg_bytes_per_launch": bpe * B,
                         "alg_bytes_per_env_step": bpe,
                         "timing": "one event pair on the launch stream around the K launches / K"},
        }
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = step_cpu_baseline(venv, acts, args.cpu_budget)
    venv.close()
    return out


def step_cpu_baseline(venv, acts, budget_s, n=4096):
    """The oracle's step() restatement (oracle/mgdp_oracle.c orc_step_batch, 1 thread) over the first
    n envs of the same batch with the same action stream, for about budget_s seconds."""
    from oracle import oracle

    st = venv.get_state()  # grids/agents as left by the timed run: same distribution of states
    ob = oracle.OracleBatch(st["enc"][:n], st["agent"][:n], venv.max_steps, venv.see_through, venv.view)
    A = acts[:, :n].cpu().numpy()
    steps = 0
    t0 = time.perf_counter()
    while True:
        ob.step(A[steps % len(A)])
        steps += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return {"value": steps * n / el, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"{steps} batched steps of {n} envs of the same workload (same action stream), "
                      f"oracle/mgdp_oracle.c orc_step_batch, {el:.1f} s"}


def gen_bench(args, rank, world, local, dist, red_dev):
    """reset(seed) for B consecutive seeds generated on the GPU (one
    gen_grids_kernel launch: seeding + the family's _gen_grid), written to device buffers; grids/s."""
    import torch

    from minigrid_dynamicprogramming_amd import gen, make

    spec = GEN_WORKLOADS[args.workload]
    B = spec["per_gpu"]
    env = make(spec["env_id"])
    W, H = env.width, env.height
    dev = torch.device("cuda", local)
    enc = torch.empty((B, W, H, 3), dtype=torch.uint8, device=dev)
    cells = torch.empty((B, H, W), dtype=torch.uint8, device=dev)
    agent = torch.empty((B, 3), dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(device=dev)

    def launch(i):
        gen.generate_device(env, rank * B, B, enc, cells, agent, device=local, stream=stream.cuda_stream)

    torch.cuda.synchronize()
    elapsed, kern_s = _timed_launches(args, launch, dist, stream)
    assert int(agent[:, 2].min().item()) >= 0, "generator reported a placement failure"
    elapsed_max, total = _max_over_ranks(dist, red_dev, elapsed, float(B) * args.steps)
    out = None
    if rank == 0:
        bpg = W * H * 3 + H * W + 12  # written per grid: encoding + type codes + agent
        avg = kern_s / args.steps
        ach = bpg * B / avg / 1e9
        out = {
            "metric": "batched reset(seed) grid generation, grids/sec, " + spec["env_id"],
            "value": total / elapsed_max, "unit": "grids/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed_max * 1000.0 / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64",
            "data": f"seeds [{rank * B}, {rank * B + B}) per rank (numpy SeedSequence/PCG64 restated in HIP)",
            "config": {"workload": args.workload, "env_id": spec["env_id"], "grids_per_gpu": B,
                       "global_grids": B * world, "parallelism": f"seed ranges x{world}"},
            "roofline": {"bound": "hbm", "kernel": "gen_grids_kernel", "achieved": ach, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                         "traffic": load_traffic(f"{args.workload}/gen", 1.0, grids=B), "launches": args.steps,
                         "avg_launch_us": avg * 1e6, "alg_bytes_per_launch": bpg * B, "alg_bytes_per_grid": bpg,
                         "regime": "integer RNG / rejection-loop latency bound (one thread per seed); "
                                   "HBM carries only the output"},
        }
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = gen_cpu_baseline(env, args.cpu_budget)
    return out


def gen_cpu_baseline(env, budget_s):
    """The host generator (minigrid_dynamicprogramming_amd/envs.py, the numpy restatement of the
    reference's reset/_gen_grid with the same Generator calls), 1 thread, seeds 0.. for budget_s."""
    n = 0
    t0 = time.perf_counter()
    while True:
        env.generate(seed=n)
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    return {"value": n / el, "unit": "grids/s", "cores": 1, "kind": "port",
            "sample": f"{n} host reset(seed) generations (numpy PCG64, envs.py), {el:.1f} s"}


BLOCK_CPU_S = 2.0  # seconds of oracle sampling per BASELINE-config block (1 thread, then all cores)
FRESH_SETS = 3  # fresh grid sets per BASELINE-config block: first-solve timing (MGDP_BENCH_FRESH overrides)
FRESH_SETS = int(os.environ.get("MGDP_BENCH_FRESH", FRESH_SETS))
# steady-state priming of a resident lone-grid server (measure(): the stated criterion)
PRIME_MIN_S, PRIME_WIN, PRIME_TOL, PRIME_MAX_S, PRIME_RELAUNCH = 0.2, 512, 0.02, 1.0, 16
PRIME_BLOCK_S = 0.03  # warmup time of each BASELINE-config block (round 6)
VALU_PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9  # MI355X_MICROARCH.md: 4 SIMD-32 per CU, one wave64 VALU op per 2 cycles


def load_sq(key):
    """Per-launch SQ counters of a kernel from the committed PMC passes (profiles/sq_counters.json,
    tools/pmc_sq.sh): VALU / LDS instructions, wave cycles, busy cycles."""
    p = os.path.join(ROOT, "profiles", "sq_counters.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f).get(key)


def hbm_side_measurement(args, n_solves=3):
    """Both batched kernels on SURVEY 8(d) config R (Empty-16x16 x 65536: 537 MB of fp32 V > the
    256 MB MALL).  `frac` is an HBM fraction of MEASURED bytes (PMC traffic per launch, else the
    kernel's compulsory bytes per launch) -- never the algorithmic figure, which counts every
    LDS-served neighbour gather as an HBM read and is reported apart as alg_equiv_gbs."""
    import torch

    import minigrid_dynamicprogramming_amd as mg

    cells, _ = make_cells(WORKLOADS["empty16x65536"], 0, 1)
    res = {}
    tsize = 4 if args.dtype == "f32" else 8
    for method in ("sweep", "fused"):
        vi = mg.ValueIteration(cells, gamma=args.gamma, tol=args.tol, dtype=args.dtype, method=method,
                               mapping=args.mapping)
        vi.solve()
        vi.enable_timing(True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ks = [vi.solve() for _ in range(n_solves)]
        el = time.perf_counter() - t0
        ms, n = vi.kernel_time()
        upd = vi.updates_per_sweep * sum(ks)
        bpu = algorithmic_bytes_per_update(tsize, 7)
        avg = ms / 1000.0 / max(n, 1)
        info = {"B": vi.B, "S": vi.S, "W": vi.W, "H": vi.H}
        if method == "sweep":  # one timed launch per sweep (the pi pass is not timed)
            comp = compulsory_bytes_per_sweep(vi.S, vi.W * vi.H, tsize) * vi.B
        else:  # V lives in LDS between sweeps: a solve's compulsory bytes, spread over its launches
            comp = compulsory_bytes_per_solve(info, tsize, "fused", ks[-1]) * n_solves / max(n, 1)
        key = f"empty16x65536/{method}/{args.mapping}/{args.dtype}"
        traffic = load_traffic(key, n_solves / max(n, 1), grids=vi.B)
        meas = traffic if traffic else comp
        r = {"kernel": vi.kernel_name, "updates_per_s": upd / el, "sweeps": ks[-1], "launches": n,
             "avg_launch_us": avg * 1e6, "bound": "hbm" if method == "sweep" else "valu/lds (not hbm)",
             "achieved": meas / avg / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": meas / avg / 1e9 / HBM_PEAK_GBS, "achieved_basis": "pmc traffic" if traffic else "compulsory bytes",
             "traffic": traffic, "compulsory_bytes_per_launch": comp,
             "compulsory_frac": comp / avg / 1e9 / HBM_PEAK_GBS,
             "alg_equiv_gbs": upd * bpu / max(n, 1) / avg / 1e9,
             "alg_note": "SURVEY 8(d) algorithmic bytes / launch time: every neighbour gather counted as an HBM "
                         "read although LDS serves it; an equivalent rate, not an HBM fraction"}
        sq = load_sq(f"{key}/{vi.kernel_name}")
        if sq and sq.get("valu_insts_per_launch"):
            lane_ops = sq["valu_insts_per_launch"] * 64.0 / avg
            r["valu"] = {"achieved": lane_ops, "peak": VALU_PEAK_LANE_OPS, "unit": "lane-ops/s",
                         "frac": lane_ops / VALU_PEAK_LANE_OPS, "source": sq.get("source")}
            if sq.get("lds_insts_per_launch"):
                r["lds_insts_per_launch"] = sq["lds_insts_per_launch"]
        res[method] = r
        vi.close()
    res["workload"] = "empty16x65536"
    return res


if __name__ == "__main__":
    main()
