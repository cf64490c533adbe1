"""Cold-start trajectory of the lone-grid (Empty-16x16, served) solve latency on a fresh box.

Phases (each solve timed on the host; per-window medians printed as JSON lines):
  cold      lone solves from the first one, for --cold-s seconds
  idle      sleep --idle-s, then lone solves for 1 s (does an idle gap cool the device again?)
  heavy     LavaS11N5 x 65536 batched solves for --heavy-s seconds
  after     lone solves for --after-s seconds right after the heavy load
  rest      sleep 5 s, lone solves for 1 s
A background thread samples the GPU's current shader / memory / fabric clock levels from sysfs
(pp_dpm_sclk / pp_dpm_mclk / pp_dpm_fclk, the '*' line) every 20 ms when they are readable.  With
MGDP_LIB pointing at a -DMGDP_SERVE_TRACE build the library also prints, per 1000 solves, the
GPU-side solve time and the shader clock from s_memtime / s_memrealtime.
"""
import argparse
import glob
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
T0 = time.perf_counter()


def now_ms():
    return (time.perf_counter() - T0) * 1e3


def find_sysfs():
    for dev in sorted(glob.glob("/sys/class/drm/card*/device")):
        p = os.path.join(dev, "pp_dpm_sclk")
        try:
            with open(p) as f:
                f.read()
            return dev
        except OSError:
            continue
    return None


def cur_level(path):
    try:
        with open(path) as f:
            for line in f:
                if line.rstrip().endswith("*"):
                    return line.split(":", 1)[1].strip().rstrip("*").strip()
    except OSError:
        return None
    return None


def sampler(dev, out, stop):
    while not stop.is_set():
        out.append((round(now_ms(), 1), *(cur_level(os.path.join(dev, f"pp_dpm_{c}")) for c in ("sclk", "mclk", "fclk", "socclk"))))
        time.sleep(0.02)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cold-s", type=float, default=3.0)
    ap.add_argument("--idle-s", type=float, default=2.0)
    ap.add_argument("--heavy-s", type=float, default=1.0)
    ap.add_argument("--after-s", type=float, default=3.0)
    ap.add_argument("--window-ms", type=float, default=25.0)
    ap.add_argument("--out", default="probe_cold.json")
    args = ap.parse_args()

    import minigrid_dynamicprogramming_amd as mg
    from minigrid_dynamicprogramming_amd import _lib

    pinned = _lib.pin_host_thread(0)
    dev = find_sysfs()
    samples, stop = [], threading.Event()
    th = None
    if dev:
        th = threading.Thread(target=sampler, args=(dev, samples, stop), daemon=True)
        th.start()
    env = mg.make("MiniGrid-Empty-16x16-v0")
    enc, _ = env.generate(seed=0)
    one = np.ascontiguousarray(enc[..., 0].T)[None]
    vi = mg.ValueIteration(one, dtype="f32")
    res = {"pinned": pinned, "sysfs": dev, "t_setup_ms": now_ms(), "phases": {}}

    def lone(name, secs):
        lat, ts = [], []
        t_end = time.perf_counter() + secs
        while time.perf_counter() < t_end:
            a = time.perf_counter()
            k = vi.solve()
            b = time.perf_counter()
            lat.append((b - a) * 1e6)
            ts.append((a - T0) * 1e3)
        assert k == 29, k
        lat, ts = np.array(lat), np.array(ts)
        wins = []
        w0 = ts[0]
        while w0 <= ts[-1]:
            m = (ts >= w0) & (ts < w0 + args.window_ms)
            if m.any():
                wins.append([round(float(w0), 1), int(m.sum()), round(float(np.median(lat[m])), 3), round(float(lat[m].mean()), 3)])
            w0 += args.window_ms
        ph = {"t_start_ms": round(float(ts[0]), 1), "n": len(lat), "first20_us": [round(x, 2) for x in lat[:20]],
              "median_us": float(np.median(lat)), "mean_us": float(lat.mean()),
              "last1000_median_us": float(np.median(lat[-1000:])), "windows[t_ms,n,median,mean]": wins}
        res["phases"][name] = ph
        print(json.dumps({name: {k: v for k, v in ph.items() if not k.startswith("windows")}}), flush=True)

    lone("cold", args.cold_s)
    vi.synchronize()
    time.sleep(args.idle_s)
    lone("after_idle", 1.0)
    vi.synchronize()
    # heavy: the batched LavaS11N5 x 65536 solve (config 4 on one GPU)
    from minigrid_dynamicprogramming_amd import gen

    lenv = mg.make("MiniGrid-LavaCrossingS11N5-v0")
    cells = gen.generate(lenv, 0, 65536, enc=False, cells=True, agent=False)["cells"]
    big = mg.ValueIteration(cells, dtype="f32")
    t_end = time.perf_counter() + args.heavy_s
    n = 0
    ta = now_ms()
    while time.perf_counter() < t_end:
        big.solve()
        n += 1
    res["phases"]["heavy"] = {"t_start_ms": ta, "solves": n, "ms_per_solve": (now_ms() - ta) / n}
    print(json.dumps({"heavy": res["phases"]["heavy"]}), flush=True)
    big.close()
    lone("after_heavy", args.after_s)
    vi.synchronize()
    time.sleep(5.0)
    lone("rest5s", 1.0)
    vi.close()
    stop.set()
    if th:
        th.join()
    res["clock_samples[t_ms,sclk,mclk,fclk,socclk]"] = samples
    with open(args.out, "w") as f:
        json.dump(res, f)
    print("done", flush=True)


if __name__ == "__main__":
    main()
