"""Does step i+1's encode overlap step i's decode? (design tool)

    python tools/overlap_probe.py [--size 256] [--dtype float32 --rate 8]     # GPU box

Times K encode+decode steps of bench.py's workload captured as hipGraphs in
two schedules: serial (one stream, encode then decode) and pipelined (encode
on stream A into one of two stream buffers, decode on stream B; step i+1's
encode starts while step i's decode runs, and step i+2's encode waits for
step i's decode to finish reading its buffer).  Checks that both schedules
leave the same decoded array as a plain encode + decode.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import cuzfp_amd as cz
    from cuzfp_amd.datagen import polynomial_field
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=256)
    p.add_argument("--dtype", default="float32")
    p.add_argument("--rate", type=float, default=8)
    p.add_argument("--steps", type=int, default=20)
    a = p.parse_args()
    shape = (a.size,) * 3
    arr = polynomial_field(shape, a.dtype)
    x = torch.from_numpy(arr).cuda()
    mb = cz.rate_to_maxbits(a.rate, arr.dtype, 3)
    w0 = cz.encode(x, mb)
    ref = cz.decode(w0, shape, x.dtype, mb)
    w = [w0, torch.empty_like(w0)]
    y = torch.empty_like(ref)
    K = a.steps
    main_s = torch.cuda.current_stream()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()

    def serial():
        for _ in range(K):
            cz.encode(x, mb, out=w[0])
            cz.decode(w[0], shape, x.dtype, mb, out=y)

    def pipelined():
        # fork from the capture stream, join back at the end
        sa.wait_stream(main_s)
        sb.wait_stream(main_s)
        enc_done = [torch.cuda.Event() for _ in range(K)]
        dec_done = [torch.cuda.Event() for _ in range(K)]
        for i in range(K):
            with torch.cuda.stream(sa):
                if i >= 2:
                    sa.wait_event(dec_done[i - 2])  # buffer i % 2 was read by decode i-2
                cz.encode(x, mb, out=w[i % 2], stream=sa)
                enc_done[i].record(sa)
            with torch.cuda.stream(sb):
                sb.wait_event(enc_done[i])
                cz.decode(w[i % 2], shape, x.dtype, mb, out=y, stream=sb)
                dec_done[i].record(sb)
        main_s.wait_stream(sa)
        main_s.wait_stream(sb)

    # eager (no graph) timing of both schedules: the GPU time per step (~50 us)
    # is well above the launch cost of two kernels and a few events
    def eager(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) / K * 1e6)
        return best
    for name, fn in (("serial", serial), ("pipelined", pipelined)):
        y.zero_()
        us = eager(fn)
        ok = bool(torch.equal(y, ref))
        print(f"eager {name:10s} wall {us:7.2f} us/step  decoded == reference: {ok}", flush=True)
    graphs = {}
    for name, fn in (("serial", serial), ("pipelined", pipelined)):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        graphs[name] = g
    for name, g in graphs.items():
        y.zero_()
        g.replay()
        torch.cuda.synchronize()
        print(f"{name}: decoded == reference: {bool(torch.equal(y, ref))}", flush=True)
    # warm the clocks, then alternate
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        graphs["serial"].replay()
        torch.cuda.synchronize()
    res = {n: [] for n in graphs}
    for _ in range(15):
        for name, g in graphs.items():
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / K * 1e6
            res[name].append((e0.elapsed_time(e1) / K * 1e3, wall))
    nbytes = x.numel() * x.element_size()
    for name, r in res.items():
        ev = sorted(t for t, _ in r)[len(r) // 2]
        wl = sorted(t for _, t in r)[len(r) // 2]
        print(f"{name:10s} events {ev:7.2f} us/step  wall {wl:7.2f} us/step  -> {nbytes / wl / 1e3:8.1f} GB/s (wall)",
              flush=True)


if __name__ == "__main__":
    main()
