"""Run the host pipeline a few times for a rocprofv3 timeline (design tool, GPU box).

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d OUT -o run -- python tools/host_trace.py
    python tools/host_trace.py --analyse OUT

The first form runs 256^3 f32 rate 8 compress_host / decompress_host from
pinned buffers (3 each after a warm-up, with 2 ms idle gaps between calls so
the calls separate in the trace); the second prints, per call, each copy and
kernel as start / end offsets from the call's first operation (us), and the
gaps on the binding copy queue.
"""
from __future__ import annotations

import csv
import glob
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run():
    import torch
    import cuzfp_amd as cz
    # --streams N: N torch streams used before the pipeline creates its own
    nst = int(sys.argv[sys.argv.index("--streams") + 1]) if "--streams" in sys.argv else 0
    keep = []
    for _ in range(nst):
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            keep.append(torch.ones(16, device="cuda") * 2)
        keep.append(st)
    torch.cuda.synchronize()
    from cuzfp_amd.datagen import polynomial_field
    arr = polynomial_field((256,) * 3, np.float32)
    mb = cz.rate_to_maxbits(8, np.float32, 3)
    h_in = torch.from_numpy(arr).pin_memory().numpy()
    s = torch.empty(cz.stream_bytes(arr.shape, arr.dtype, mb) // 8, dtype=torch.int64).pin_memory().numpy().view(np.uint64)
    y = torch.empty(arr.shape, dtype=torch.float32).pin_memory().numpy()
    cz.compress_host(h_in, mb, out=s)
    cz.decompress_host(s, arr.shape, np.float32, mb, out=y)
    for _ in range(3):
        time.sleep(0.002)
        cz.compress_host(h_in, mb, out=s)
    for _ in range(3):
        time.sleep(0.002)
        cz.decompress_host(s, arr.shape, np.float32, mb, out=y)
    print("ok")


def analyse(root):
    ev = []
    for f in glob.glob(os.path.join(root, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", "copy"),
                       int(r.get("Bytes", 0) or 0)))
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "zfp_" in r["Kernel_Name"]:
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                           "enc" if "encode" in r["Kernel_Name"] else "dec", 0))
    ev.sort()
    calls, cur = [], []
    for e in ev:  # split at idle gaps > 1 ms
        if cur and e[0] - max(x[1] for x in cur) > 1_000_000:
            calls.append(cur)
            cur = []
        cur.append(e)
    if cur:
        calls.append(cur)
    for c in calls:
        t0 = c[0][0]
        span = (max(x[1] for x in c) - t0) / 1e3
        print(f"call: {span:8.1f} us, {len(c)} ops")
        for s, e, kind, b in c:
            print(f"   {kind:18s} {(s - t0) / 1e3:8.1f} .. {(e - t0) / 1e3:8.1f}  ({(e - s) / 1e3:7.1f} us"
                  + (f", {b / 2**20:6.2f} MiB, {b / (e - s):6.2f} GB/s)" if b else ")"))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyse":
        analyse(sys.argv[2])
    else:
        run()
