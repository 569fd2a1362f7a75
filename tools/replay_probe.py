"""How the timed region's numbers depend on what runs before it (design tool).

  python tools/replay_probe.py        # GPU box

Captures bench.py's step (encode + decode of the 256^3 f32 array at rate 8)
as one hipGraph of 20 steps and times consecutive replays, each between two
synchronizes (wall clock) and with HIP events: after a cold start, after the
GPU idled, and with the replays back to back.
"""
from __future__ import annotations

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
    a = polynomial_field((256,) * 3, np.float32)
    x = torch.from_numpy(a).cuda()
    mb = cz.rate_to_maxbits(8, np.float32, 3)
    w = cz.encode(x, mb)
    y = cz.decode(w, a.shape, x.dtype, mb)

    def step():
        cz.encode(x, mb, out=w)
        cz.decode(w, a.shape, x.dtype, mb, out=y)

    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20):
            step()
    s = torch.cuda.current_stream()

    def timed(label):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(s)
        g.replay()
        e1.record(s)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / 20 * 1e6
        print(f"{label:28s} wall {wall:6.2f} us/step  events {e0.elapsed_time(e1) / 20 * 1e3:6.2f} us/step",
              flush=True)

    for i in range(4):
        timed(f"cold, replay {i}")
    time.sleep(0.5)
    timed("after 0.5 s idle")
    timed("next")
    # 100 ms of back-to-back replays, then timed replays
    for _ in range(100):  # ~100 ms of GPU work
        g.replay()
    for i in range(4):
        timed(f"after 100 ms busy, {i}")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    for _ in range(10):
        g.replay()
    e1.record(s)
    torch.cuda.synchronize()
    print(f"{'10 replays back to back':28s} events {e0.elapsed_time(e1) / 200 * 1e3:6.2f} us/step", flush=True)

    # the same 20 steps as eager launches straight through the C-ABI (ctypes,
    # arguments prepared once), after keeping the GPU busy
    import ctypes
    lib = cz.library()
    t, ex = cz.type_code(x.dtype), cz._extents(x.shape)
    st = ctypes.c_void_p(s.cuda_stream)
    nb = ctypes.c_size_t(w.numel() * 8)
    got = ctypes.c_size_t(0)
    enc_args = (ctypes.c_void_p(x.data_ptr()), t, *ex, 0, 0, 0, mb, ctypes.c_void_p(w.data_ptr()), nb,
                ctypes.byref(got), st)
    dec_args = (ctypes.c_void_p(w.data_ptr()), nb, t, *ex, 0, 0, 0, mb, ctypes.c_void_p(y.data_ptr()), st)
    enc, dec = lib.cuzfp_hip_encode, lib.cuzfp_hip_decode

    def eager20():
        for _ in range(20):
            enc(*enc_args)
            dec(*dec_args)

    for i in range(3):
        for _ in range(100):
            g.replay()
        torch.cuda.synchronize()
        e0.record(s)
        t0 = time.perf_counter()
        eager20()
        e1.record(s)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / 20 * 1e6
        print(f"{'eager ctypes after busy':28s} wall {wall:6.2f} us/step  events {e0.elapsed_time(e1) / 20 * 1e3:6.2f} us/step", flush=True)
        for _ in range(100):
            g.replay()
        timed("graph after busy")


if __name__ == "__main__":
    main()
