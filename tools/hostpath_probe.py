"""Why bench.py's host_path and tools/host_sweep.py disagree (design tool, GPU box).

    python tools/hostpath_probe.py

Times compress_host / decompress_host of the 256^3 f32 array from pinned
buffers in one process, the way each tool does it (buffers made as the tool
makes them, its timing loop), before and after a burst of device-resident codec
launches like the bench's timed region.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import cuzfp_amd as cz
    # --streams N: create N torch streams (and run a kernel on each) before the
    # pipeline creates its own, as a process that has used streams already has
    nst = int(sys.argv[sys.argv.index("--streams") + 1]) if "--streams" in sys.argv else 0
    keep = []
    for _ in range(nst):
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            keep.append(torch.ones(16, device="cuda") * 2)
        keep.append(st)
    torch.cuda.synchronize()
    from cuzfp_amd.datagen import polynomial_field
    a = polynomial_field((256,) * 3, np.float32)
    mb = cz.rate_to_maxbits(8, np.float32, 3)
    sb = cz.stream_bytes(a.shape, a.dtype, mb)
    # bench.py's buffers
    b_in = torch.from_numpy(a).pin_memory().numpy()
    b_out = torch.empty(sb // 8, dtype=torch.int64).pin_memory().numpy().view(np.uint64)
    b_back = torch.empty(a.shape, dtype=torch.float32).pin_memory().numpy()
    # host_sweep.py's buffers (tensors kept)
    t_in = torch.from_numpy(a).pin_memory()
    t_s = torch.empty(sb // 8, dtype=torch.int64).pin_memory()
    t_out = torch.empty(a.shape, dtype=torch.float32).pin_memory()

    def med(fn, n=7, sync=False):
        fn()
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            if sync:
                torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return round(a.nbytes / ts[len(ts) // 2] / 1e9, 2), [round(t * 1e6) for t in ts]

    def report(tag):
        r = {}
        r["bench_bufs_compress"] = med(lambda: cz.compress_host(b_in, mb, out=b_out))
        r["bench_bufs_decompress"] = med(lambda: cz.decompress_host(b_out, a.shape, np.float32, mb, out=b_back))
        s_np = t_s.numpy().view(np.uint64)
        r["sweep_bufs_compress"] = med(lambda: cz.compress_host(t_in.numpy(), mb, out=s_np), sync=True)
        r["sweep_bufs_decompress"] = med(lambda: cz.decompress_host(s_np, a.shape, np.float32, mb, out=t_out.numpy()),
                                         sync=True)
        print(tag, json.dumps(r), flush=True)

    report(f"fresh, {nst} streams before")
    x = torch.from_numpy(a).cuda()
    w = cz.encode(x, mb)
    y = cz.decode(w, a.shape, x.dtype, mb)
    for _ in range(200):
        cz.encode(x, mb, out=w)
        cz.decode(w, a.shape, x.dtype, mb, out=y)
    torch.cuda.synchronize()
    report("after device codec")


if __name__ == "__main__":
    main()
