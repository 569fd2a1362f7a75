"""Per-copy cost of chunked pinned transfers (design tool, GPU box).

    python tools/copy_chunks.py [--mib 64]

The host pipeline (capi.hip host_pipeline) moves an array in chunks with an
event after each copy and cross-stream waits between the copies and the
kernels.  The round-5 sweep (tools/host_sweep.py) priced that at ~20 us a
chunk.  This times the pieces on their own, through the HIP runtime (ctypes),
so the pipeline's shape can be chosen from what each piece costs:
  one copy of the whole buffer, k back-to-back copies on one stream, the same
  with an event recorded after each, with a second stream waiting on each
  event, and H2D beside D2H (full duplex).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import time


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=64)
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    hip = ctypes.CDLL("libamdhip64.so")
    vp, sz = ctypes.c_void_p, ctypes.c_size_t

    def ok(e):
        assert e == 0, e

    nbytes = a.mib << 20
    h = vp()
    ok(hip.hipHostMalloc(ctypes.byref(h), sz(nbytes), 0))
    h2 = vp()
    ok(hip.hipHostMalloc(ctypes.byref(h2), sz(nbytes), 0))
    d = vp()
    ok(hip.hipMalloc(ctypes.byref(d), sz(nbytes)))
    d2 = vp()
    ok(hip.hipMalloc(ctypes.byref(d2), sz(nbytes)))
    ctypes.memset(h, 1, nbytes)
    st = [vp() for _ in range(3)]
    for s in st:
        ok(hip.hipStreamCreateWithFlags(ctypes.byref(s), 1))
    evs = [vp() for _ in range(256)]
    for e in evs:
        ok(hip.hipEventCreateWithFlags(ctypes.byref(e), 2))  # disable timing
    H2D, D2H = 1, 2

    def copies(k, kind, stream, events=False, waiter=None, dst=None, src=None):
        c = nbytes // k
        for i in range(k):
            off = i * c
            if kind == H2D:
                ok(hip.hipMemcpyAsync(vp((dst or d).value + off), vp((src or h).value + off), sz(c), H2D, stream))
            else:
                ok(hip.hipMemcpyAsync(vp((dst or h2).value + off), vp((src or d).value + off), sz(c), D2H, stream))
            if events:
                ok(hip.hipEventRecord(evs[i], stream))
                if waiter is not None:
                    ok(hip.hipStreamWaitEvent(waiter, evs[i], 0))

    def timed(fn):
        fn()
        ok(hip.hipDeviceSynchronize())
        ts = []
        for _ in range(a.reps):
            t = time.perf_counter()
            fn()
            ok(hip.hipDeviceSynchronize())
            ts.append(time.perf_counter() - t)
        ts.sort()
        return ts[len(ts) // 2]

    res = {}
    for kind, name in ((H2D, "h2d"), (D2H, "d2h")):
        for k in (1, 4, 8, 16, 64):
            t0 = timed(lambda: copies(k, kind, st[0]))
            t1 = timed(lambda: copies(k, kind, st[0], events=True))
            t2 = timed(lambda: copies(k, kind, st[0], events=True, waiter=st[1]))
            r = {"chunks": k, "plain_GBps": round(nbytes / t0 / 1e9, 2), "events_GBps": round(nbytes / t1 / 1e9, 2),
                 "waited_GBps": round(nbytes / t2 / 1e9, 2)}
            res[f"{name}_{k}"] = r
            print(name, json.dumps(r), flush=True)
    # the same chunks alternating between two streams (two copy engines), so
    # that one copy's own cost overlaps the other's transfer
    def copies2(k, kind):
        c = nbytes // k
        for i in range(k):
            off = i * c
            s = st[i % 2]
            if kind == H2D:
                ok(hip.hipMemcpyAsync(vp(d.value + off), vp(h.value + off), sz(c), H2D, s))
            else:
                ok(hip.hipMemcpyAsync(vp(h2.value + off), vp(d.value + off), sz(c), D2H, s))
    for kind, name in ((H2D, "h2d"), (D2H, "d2h")):
        for k in (4, 8, 16):
            t = timed(lambda: copies2(k, kind))
            res[f"{name}_{k}_two_streams_GBps"] = round(nbytes / t / 1e9, 2)
            print(name, k, "chunks on two streams", res[f"{name}_{k}_two_streams_GBps"], flush=True)
    # full duplex: H2D on stream 0 beside D2H on stream 2, the whole buffer each
    t = timed(lambda: (copies(1, H2D, st[0]), copies(1, D2H, st[2], src=d2)))
    res["duplex_each_GBps"] = round(nbytes / t / 1e9, 2)
    print("duplex (H2D beside D2H, each direction)", res["duplex_each_GBps"], flush=True)
    t = timed(lambda: (copies(16, H2D, st[0], events=True), copies(16, D2H, st[2], events=False, src=d2)))
    res["duplex16_each_GBps"] = round(nbytes / t / 1e9, 2)
    print("duplex, 16 chunks each", res["duplex16_each_GBps"], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
