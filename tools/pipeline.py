"""Encode+decode round trips pipelined over two HIP streams (design tool, GPU
box): the decode of round trip k on one stream while the encode of round trip
k+1 runs on the other, streams double-buffered.  Microseconds per round trip.

  python tools/pipeline.py [--size S] [--steps K]

  serial        one stream, hipGraph of K round trips (the bench's step)
  pipe-graph    two streams captured into one hipGraph
  pipe-eager    two streams, eager launches
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--only", default="", help="comma-separated variant names")
    a = ap.parse_args()
    import torch
    import cuzfp_amd as cz
    from cuzfp_amd.datagen import polynomial_field
    shape = (a.size,) * 3
    x = torch.from_numpy(polynomial_field(shape)).cuda()
    mb = cz.rate_to_maxbits(8, x.cpu().numpy().dtype, 3)
    ref = cz.encode(x, mb)
    w = [torch.empty_like(ref), torch.empty_like(ref)]
    y = torch.empty_like(x)
    K = a.steps
    sB = torch.cuda.Stream()

    def serial():
        for _ in range(K):
            cz.encode(x, mb, out=w[0])
            cz.decode(w[0], shape, x.dtype, mb, out=y)

    def pipelined_on(sA, sB):
        # E_k on A; D_k on B after E_k; E_{k+2} (same buffer) after D_k
        cur = torch.cuda.current_stream()
        sA.wait_stream(cur)
        sB.wait_stream(cur)
        done = [None, None]
        for k in range(K):
            b = k & 1
            if done[b] is not None:
                sA.wait_event(done[b])
            with torch.cuda.stream(sA):
                cz.encode(x, mb, out=w[b])
            ev = torch.cuda.Event()
            ev.record(sA)
            sB.wait_event(ev)
            with torch.cuda.stream(sB):
                cz.decode(w[b], shape, x.dtype, mb, out=y)
            d = torch.cuda.Event()
            d.record(sB)
            done[b] = d
        cur.wait_stream(sA)
        cur.wait_stream(sB)

    def pipelined():  # the capture stream under a graph carries the encodes
        pipelined_on(torch.cuda.current_stream(), sB)

    # stream priorities (lower number = higher priority): the decodes' queue
    # ahead of the encodes', so that decode k's workgroups are all dispatched
    # before encode k+1's, which then take the slots decode k's waves free
    lo, hi = torch.cuda.Stream(priority=0), torch.cuda.Stream(priority=-1)
    lo2, hi2 = torch.cuda.Stream(priority=0), torch.cuda.Stream(priority=-1)

    def graphed(fn):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        return g.replay

    variants = {"serial": graphed(serial), "pipe-eager": pipelined,
                "pipe-prio-dec": lambda: pipelined_on(lo, hi),
                "pipe-prio-enc": lambda: pipelined_on(hi2, lo2)}
    if a.only:
        variants = {k: v for k, v in variants.items() if k in a.only.split(",")}
    try:
        if not a.only or "pipe-graph" in a.only.split(","):
            variants["pipe-graph"] = graphed(pipelined)
    except Exception as e:  # pragma: no cover
        print("pipe-graph capture failed:", e)
    res = {}
    for name, fn in variants.items():
        fn()
        torch.cuda.synchronize()
        r = []
        for _ in range(7):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                fn()
            e1.record()
            torch.cuda.synchronize()
            r.append(e0.elapsed_time(e1) / (3 * K) * 1000)
        res[name] = round(sorted(r)[3], 2)
        print(f"{name:11s} {res[name]:8.2f} us per round trip", flush=True)
    # the pipelined round trips decode to the same array
    for f in (pipelined_on,):
        w[0].zero_(); w[1].zero_(); y.zero_()
        f(lo, hi)
        torch.cuda.synchronize()
        assert torch.equal(w[0], ref) and torch.equal(w[1], ref)
        assert torch.equal(y, cz.decode(ref, shape, x.dtype, mb))
    print("pipelined round trips: streams and decode == serial")
    assert torch.equal(w[0], ref) and torch.equal(w[1], ref)
    assert torch.equal(y, cz.decode(ref, shape, x.dtype, mb))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
