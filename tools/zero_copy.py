"""The codec kernels reading / writing pinned host memory directly (design tool, GPU box).

    python tools/zero_copy.py [--size 256]

The host pipeline (capi.hip host_pipeline) moves chunks with DMA copies, and
every copy costs ~10-15 us of its own (tools/copy_chunks.py).  A kernel can
instead load and store pinned host memory itself over PCIe (the buffer
mapped into the device's address space by hipHostMalloc).  This times, for
the 256^3 f32 array at rate 8 from hipHostMalloc buffers:
  the copy kernel (cuzfp_hip_copy) host -> device and device -> host,
  the encoder reading the host array (stream to device memory, and to host),
  the decoder reading the host stream and writing the host array,
beside the DMA link (one hipMemcpyAsync of the whole buffer), and checks that
the streams and arrays match the device-resident codec's bytes.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--ranges", action="store_true", help="only probe the pinned-pointer queries")
    a = ap.parse_args()
    import cuzfp_amd as cz
    from cuzfp_amd.datagen import polynomial_field
    hip = ctypes.CDLL("libamdhip64.so")
    lib = cz.library()
    vp, sz = ctypes.c_void_p, ctypes.c_size_t

    def ok(e):
        assert e == 0, e

    arr = polynomial_field((a.size,) * 3, np.float32)
    n = arr.nbytes
    mb = cz.rate_to_maxbits(8, np.float32, 3)
    sb = cz.stream_bytes(arr.shape, arr.dtype, mb)

    def host(nbytes):
        p = vp()
        ok(hip.hipHostMalloc(ctypes.byref(p), sz(nbytes), 0))
        d = vp()
        ok(hip.hipHostGetDevicePointer(ctypes.byref(d), p, 0))
        assert d.value == p.value, (hex(p.value), hex(d.value))  # one address on host and device
        return p

    def dev(nbytes):
        p = vp()
        ok(hip.hipMalloc(ctypes.byref(p), sz(nbytes)))
        return p

    h_in, h_out, h_s = host(n), host(n), host(sb)
    d_in, d_out, d_s = dev(n), dev(n), dev(sb)
    ctypes.memmove(h_in, arr.ctypes.data, n)
    ok(hip.hipMemcpy(d_in, h_in, sz(n), 1))
    st = vp()
    ok(hip.hipStreamCreateWithFlags(ctypes.byref(st), 1))
    nx = ny = nz = a.size
    T = 3  # CUZFP_TYPE_FLOAT

    def enc(src, dst):
        ok(lib.cuzfp_hip_encode(src, T, nx, ny, nz, ctypes.c_longlong(0), ctypes.c_longlong(0), ctypes.c_longlong(0),
                                mb, dst, sz(sb), None, st))

    def dec(src, dst):
        ok(lib.cuzfp_hip_decode(src, sz(sb), T, nx, ny, nz, ctypes.c_longlong(0), ctypes.c_longlong(0),
                                ctypes.c_longlong(0), mb, dst, st))

    def timed(fn):
        fn()
        ok(hip.hipStreamSynchronize(st))
        ts = []
        for _ in range(a.reps):
            t = time.perf_counter()
            fn()
            ok(hip.hipStreamSynchronize(st))
            ts.append(time.perf_counter() - t)
        ts.sort()
        return ts[len(ts) // 2]

    res = {}
    gb = lambda t: round(n / t / 1e9, 2)
    res["dma_h2d_GBps"] = gb(timed(lambda: ok(hip.hipMemcpyAsync(d_out, h_in, sz(n), 1, st))))
    res["dma_d2h_GBps"] = gb(timed(lambda: ok(hip.hipMemcpyAsync(h_out, d_in, sz(n), 2, st))))
    res["kernel_h2d_GBps"] = gb(timed(lambda: ok(lib.cuzfp_hip_copy(h_in, d_out, sz(n), st))))
    res["kernel_d2h_GBps"] = gb(timed(lambda: ok(lib.cuzfp_hip_copy(d_in, h_out, sz(n), st))))
    print(json.dumps(res), flush=True)
    # reference bytes: the device-resident codec
    enc(d_in, d_s)
    dec(d_s, d_out)
    ok(hip.hipStreamSynchronize(st))
    ref_s = np.empty(sb // 8, np.uint64)
    ref_y = np.empty(arr.shape, np.float32)
    ok(hip.hipMemcpy(ctypes.c_void_p(ref_s.ctypes.data), d_s, sz(sb), 2))
    ok(hip.hipMemcpy(ctypes.c_void_p(ref_y.ctypes.data), d_out, sz(n), 2))
    res["device_encode_us"] = round(timed(lambda: enc(d_in, d_s)) * 1e6, 1)
    res["device_decode_us"] = round(timed(lambda: dec(d_s, d_out)) * 1e6, 1)
    t = timed(lambda: enc(h_in, d_s))
    res["encode_host_in_GBps"] = gb(t)
    t = timed(lambda: enc(h_in, h_s))
    res["encode_host_in_out_GBps"] = gb(t)
    s_host = np.ctypeslib.as_array(ctypes.cast(h_s, ctypes.POINTER(ctypes.c_uint64)), (sb // 8,))
    res["encode_host_stream_equal"] = bool(np.array_equal(s_host, ref_s))
    t = timed(lambda: dec(h_s, h_out))
    res["decode_host_in_out_GBps"] = gb(t)
    y_host = np.ctypeslib.as_array(ctypes.cast(h_out, ctypes.POINTER(ctypes.c_float)), arr.shape)
    res["decode_host_equal"] = bool(np.array_equal(y_host.view(np.uint32), ref_y.view(np.uint32)))
    t = timed(lambda: dec(d_s, h_out))
    res["decode_host_out_GBps"] = gb(t)
    print(json.dumps(res), flush=True)


if __name__ == "__main__" and "--ranges" not in sys.argv:
    main()


def probe_ranges():
    """hipMemGetAddressRange / hipHostGetDevicePointer on pinned host pointers
    (hipHostMalloc, torch's pinned allocator, hipHostRegister), at the base and inside."""
    import torch
    hip = ctypes.CDLL("libamdhip64.so")
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    out = {}
    p = vp()
    assert hip.hipHostMalloc(ctypes.byref(p), sz(1 << 20), 0) == 0
    t = torch.empty(1 << 18, dtype=torch.float32).pin_memory()
    reg = np.zeros(1 << 18, np.float32)
    rc_reg = hip.hipHostRegister(vp(reg.ctypes.data), sz(reg.nbytes), 0)
    for name, base in (("hipHostMalloc", p.value), ("torch_pinned", t.data_ptr()), ("hipHostRegister", reg.ctypes.data)):
        for off in (0, 4096 + 16):
            d = vp()
            e1 = hip.hipHostGetDevicePointer(ctypes.byref(d), vp(base + off), 0)
            b, s = vp(), sz()
            e2 = hip.hipMemGetAddressRange(ctypes.byref(b), ctypes.byref(s), d if d.value else vp(base + off))
            out[f"{name}+{off}"] = {"getdev_rc": e1, "same_addr": (d.value == base + off) if d.value else None,
                                    "range_rc": e2, "range_base_off": (b.value - base) if b.value else None,
                                    "range_size": s.value}
    out["register_rc"] = rc_reg
    print(json.dumps(out), flush=True)


if __name__ == "__main__" and "--ranges" in sys.argv:
    probe_ranges()
