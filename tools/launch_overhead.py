"""Wall-clock cost of bench.py's timed region by launch form (design tool).

    python tools/launch_overhead.py [--steps 20] [--reps 15]

bench.py times K steps (the driver runs K = 20) as wall time between a
synchronize before and after.  At K = 20 one step's kernels take ~48 us, so
a fixed launch cost of tens of microseconds is a few percent of the line.
This times the same K steps of the 256^3 f32 rate-8 step, by launch form:
  graph(K)      one hipGraph of K steps, replayed once (bench.py's form)
  graph(k)xK/k  a graph of k steps replayed K/k times
  eager         2K plain launches from Python
Each form runs `reps` times after a warm-up; the median wall time per step and
the GPU time per step (HIP events on the launch stream) are printed.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--sched", choices=["auto", "spin", "yield", "blocking"], default="auto",
                    help="hipSetDeviceFlags scheduling mode, set before the device is used")
    a = ap.parse_args()
    if a.sched != "auto":
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        rc = hip.hipSetDeviceFlags({"spin": 1, "yield": 2, "blocking": 4}[a.sched])
        print(f"hipSetDeviceFlags({a.sched}) -> {rc}", flush=True)
    import numpy as np
    import torch
    import cuzfp_amd as cz
    from cuzfp_amd.datagen import polynomial_field
    shape = (256, 256, 256)
    arr = polynomial_field(shape, np.float32)
    x = torch.from_numpy(arr).cuda()
    mb = cz.rate_to_maxbits(8, np.float32, 3)
    w = cz.encode(x, mb)
    y = cz.decode(w, shape, x.dtype, mb)
    stream = torch.cuda.current_stream()

    def step():
        cz.encode(x, mb, out=w)
        cz.decode(w, shape, x.dtype, mb, out=y)

    def graph(k):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(k):
                step()
        g.replay()
        torch.cuda.synchronize()
        return g

    K = a.steps
    forms = {}
    for k in sorted({K, 10, 5, 2, 1}, reverse=True):
        if K % k == 0:
            g = graph(k)
            forms[f"graph({k})x{K // k}"] = (lambda g=g, n=K // k: [g.replay() for _ in range(n)])
    forms["eager"] = lambda: [step() for _ in range(K)]
    # keep the GPU busy before each measurement (clocks), as bench.py does
    busy = graph(50)
    out = {}
    for name, fn in forms.items():
        walls, gpus = [], []
        for _ in range(a.reps):
            busy.replay()
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record(stream)
            fn()
            e1.record(stream)
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) / K * 1e6)
            gpus.append(e0.elapsed_time(e1) / K * 1e3)
        walls_raw = list(walls)
        walls.sort()
        gpus.sort()
        first = walls_raw[0]
        out[name] = {"wall_us_per_step": round(walls[len(walls) // 2], 2), "gpu_us_per_step": round(gpus[len(gpus) // 2], 2),
                     "wall_min": round(walls[0], 2), "wall_max": round(walls[-1], 2), "wall_first": round(first, 2)}
        print(name, out[name], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
