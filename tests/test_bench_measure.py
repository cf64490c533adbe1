"""bench.measure() end to end on the CPU: the ValueIteration handle replaced by a fake backed by the
oracle (a closed handle refuses every call, like the real one), so the warmup / priming / timed
region / result bookkeeping runs without a GPU -- the lone-grid priming rule and latency record, the
batched executed-sweeps record, no handle use after close."""
import argparse
import importlib.util
import os

import numpy as np
import pytest

from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class FakeVI:
    """The bits of dp.ValueIteration that bench.measure() uses, solved by the oracle."""

    def __init__(self, cells, gamma=0.99, tol=1e-6, dtype="f32", method="fused", mapping="cell", device=0):
        self._cells = np.ascontiguousarray(cells)
        self._open = True
        self._dtype = dtype
        self._tol = tol
        self._timing = False
        self._solves = 0
        B, H, W = self._cells.shape
        self._dims = dict(B=B, H=H, W=W, S=W * H * 4, model="xyd", updates_per_sweep=B * W * H * 4 * 7,
                          kernel_name="vi_serve_kernel" if B == 1 else "vi_fused_kernel", persistent=B == 1)
        self._own = None

    def __getattr__(self, name):
        d = self.__dict__
        if name in d.get("_dims", {}):
            if not d["_open"]:
                raise ValueError("null argument")  # what the C ABI says for a destroyed handle
            return d["_dims"][name]
        raise AttributeError(name)

    def _check(self):
        if not self._open:
            raise ValueError("null argument")

    def enable_timing(self, on=True):
        self._check()
        self._timing = on
        self._solves = 0

    def solve(self, last=False):
        self._check()
        r = oracle.value_iteration(0, self._cells, tol=self._tol, dtype=self._dtype)
        self._solves += 1
        if self._own is None:
            self._own = np.array([oracle.value_iteration(0, c, tol=self._tol, dtype=self._dtype)["sweeps"]
                                  for c in self._cells], np.int32)
        return r["sweeps"]

    def synchronize(self):
        self._check()

    def kernel_time(self):
        self._check()
        return 0.01 * self._solves, (1 if self.persistent else self._solves)

    def serve_clock(self):
        self._check()
        return {"sclk_mhz": 2400.0, "server_us": 10.0 * self._solves, "launches": 1}

    def grid_sweeps(self):
        self._check()
        return self._own

    def close(self):
        self._open = False


@pytest.fixture
def bench(monkeypatch):
    import torch

    import minigrid_dynamicprogramming_amd as mg

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    monkeypatch.setattr(mg, "ValueIteration", FakeVI)
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
    monkeypatch.setattr(b, "PRIME_MIN_S", 0.01)
    monkeypatch.setattr(b, "PRIME_WIN", 8)
    return b


def _args(workload, steps=3, warmup=2):
    return argparse.Namespace(workload=workload, steps=steps, warmup=warmup, gamma=0.99, tol=1e-6,
                              method="fused", mapping="cell")


def test_measure_lone_grid_priming_and_latency(bench):
    import minigrid_dynamicprogramming_amd as mg

    enc, _ = mg.make("MiniGrid-Empty-16x16-v0").generate(seed=0)
    cells = np.ascontiguousarray(enc[..., 0].T)[None]
    m = bench.measure(_args("empty16"), "f32", cells, 0, None, None, None, False)
    assert m["sweeps"] == [29, 29, 29] and m["upd_total"] == 29 * 3 * 1024 * 7
    lat = m["latency"]
    # whole windows, the warm server's last solve, then the relaunch priming
    n = lat["priming_solves"] - 1 - bench.PRIME_RELAUNCH
    assert n >= 2 * bench.PRIME_WIN and n % bench.PRIME_WIN == 0
    assert lat["warm_phase_clock"]["sclk_mhz"] == 2400.0
    assert len(lat["warmup_solves_us"]) == 2 and lat["first_solve_us"] > 0
    assert lat["device_clock"]["sclk_mhz"] == 2400.0 and "windows of 8" in lat["steady_rule"]
    assert m["executed"] is None and m["info"]["persistent"] is True


def test_measure_batch_executed_sweeps(bench):
    from minigrid_dynamicprogramming_amd import make

    env = make("MiniGrid-FourRooms-v0")
    cells = np.stack([np.ascontiguousarray(env.generate(seed=s)[0][..., 0].T) for s in range(6)])
    m = bench.measure(_args("fourrooms4096"), "f32", cells, 0, None, None, None, False)
    K = m["sweeps"][-1]
    ex = m["executed"]
    assert ex["global_sweeps"] == K and 0 < ex["frac_of_global_rule"] <= 1.0
    assert m["latency"] is None and m["primed"] == 0


def test_measure_split_events_pass(bench):
    # the blocks' timed region runs without per-launch events; the roofline's launch count comes
    # from the second pass of the same K solves
    from minigrid_dynamicprogramming_amd import make

    env = make("MiniGrid-FourRooms-v0")
    cells = np.stack([np.ascontiguousarray(env.generate(seed=s)[0][..., 0].T) for s in range(4)])
    m = bench.measure(_args("fourrooms4096", steps=4), "f32", cells, 0, None, None, None, False, split_events=True)
    assert m["events_in_region"] is False and m["launches"] == 4 and len(m["sweeps"]) == 4
    m = bench.measure(_args("fourrooms4096", steps=4), "f32", cells, 0, None, None, None, False)
    assert m["events_in_region"] is True


def _full_record():
    """A default-line record with every block at its longest (values with many digits)."""
    import math

    def cpu(v):
        return {"value": v * math.pi, "unit": "updates/s", "cores": 16, "kind": "port",
                "sample": "12345 full solves of 512 grid(s) of the same workload (69 sweeps in the last, f32), "
                          "oracle/mgdp_oracle.c orc_vi (literal global loop), 2.0 s"}

    def blk(v, k):
        return {"value": v * math.e, "unit": "updates/s", "ms_per_solve": 2.4938271, "sweeps": k,
                "executed_updates_per_s": v * 1.7182818, "executed_rank0": {"frac_of_global_rule": 0.62912345},
                "roofline": {"valu": {"frac": 0.41234567}}, "cpu_baseline": cpu(1e9), "cpu_baseline_all_cores": cpu(1e10),
                "cpu_baseline_fp": cpu(2e9), "cpu_baseline_fp_all_cores": cpu(2e10)}

    return {"metric": "state-action Bellman updates/sec + DP sweeps-to-converge, Empty-16x16", "value": 2.5123456789e10,
            "unit": "updates/s", "n_gpus": 8, "steps": 200, "warmup": 20, "ms_per_step": 0.00828030169941485,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: MiniGrid-Empty-16x16-v0 grids from the reference-exact generator (seed 0 replicated)",
            "config": {"workload": "empty16", "env_id": "MiniGrid-Empty-16x16-v0", "grids_per_gpu": 1, "global_grids": 8,
                       "states_per_grid": 1024, "actions": 7, "gamma": 0.99, "tol": 1e-6, "method": "fused",
                       "mapping": "cell", "parallelism": "replicas only", "host_thread": "pinned (128 CPUs)"},
            "sweeps": 29,
            "roofline": {"bound": "hbm", "kernel": "vi_serve_kernel", "achieved": 144.46552140524724, "peak": 8000.0,
                         "unit": "GB/s", "frac": 0.018058190175655905, "traffic": 63168.123, "launches": 1,
                         "avg_launch_us": 288.6030077934265, "solves_per_launch": 36.0, "note": "x" * 500},
            "cpu_baseline": cpu(1e9), "cpu_baseline_all_cores": cpu(1e10),
            "latency": {"gpu_solve_us": 6.271, "host_and_handoff_us": 2.012},
            "batched": {"fourrooms4096": blk(2.6e13, 37)},
            "sharded": {"lava65536": blk(6.6e13, 49), "doorkey65536": blk(3.7e13, 69)}}


def test_compact_line_fits_the_driver_tail(bench):
    """The stdout line keeps every contract key and one summary per BASELINE config, in < 2000 chars
    (the driver records the last 2000 characters of stdout)."""
    import json

    out = _full_record()
    txt = bench.compact_dumps(bench.compact_line(out))
    assert len(txt) < 1950, len(txt)
    c = json.loads(txt)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in c, k
    assert c["roofline"]["frac"] == pytest.approx(0.0181, rel=1e-3)
    assert c["value"] == pytest.approx(out["value"], rel=1e-5)
    assert set(c["configs"]) == {"empty16", "fourrooms4096", "lava65536", "doorkey65536"}
    fr = c["configs"]["fourrooms4096"]
    assert fr["v"] == pytest.approx(2.6e13 * 2.718281828, rel=1e-3)
    assert fr["x"] == pytest.approx(2.6e13 * 1.7182818, rel=1e-3)
    assert {"c1", "c16", "f1", "f16", "xf", "valu", "k", "ms"} <= set(fr)
