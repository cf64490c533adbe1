"""bench.py --gpus N without a torch.distributed environment starts its own N ranks (a child
torch.distributed.run, before any GPU call) and reports rank 0's line with n_gpus = N; a failing
rank makes the whole command fail.  CPU only: MGDP_BENCH_DRYRUN runs the rank plumbing over gloo."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, extra_env=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                              "MASTER_PORT")}
    env.update({"MGDP_BENCH_DRYRUN": "1", "OMP_NUM_THREADS": "1"}, **(extra_env or {}))
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "3",
                           "--warmup", "1"], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)


@pytest.mark.parametrize("n", [2, 4])
def test_self_launch_starts_n_ranks(n):
    r = _run(n)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints the line
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["ranks"] == [0, n] and out["steps"] == 3
    assert out["elapsed_max"] == pytest.approx(0.001 * n)  # the max over all ranks' regions


def test_self_launch_propagates_a_rank_failure():
    r = _run(2, {"MGDP_BENCH_DRYRUN_FAIL_RANK": "1"})
    assert r.returncode != 0


def test_single_gpu_does_not_self_launch():
    r = _run(1)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["n_gpus"] == 1 and "launching" not in r.stderr


def test_shard_of_rehearsal_knob(monkeypatch):
    # MGDP_BENCH_SHARD_OF=N (tools/gpu_shard.sh) gives a world-1 run rank 0's shard of an N-way split;
    # it never changes a real multi-rank run
    import importlib.util

    from minigrid_dynamicprogramming_amd.distributed import shard_range

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    monkeypatch.delenv("MGDP_BENCH_SHARD_OF", raising=False)
    assert bench.shard_of(1) == 1 and bench.shard_of(4) == 4
    monkeypatch.setenv("MGDP_BENCH_SHARD_OF", "8")
    assert bench.shard_of(1) == 8 and bench.shard_of(2) == 2
    assert shard_range(65536, 0, bench.shard_of(1)) == (0, 8192)
