"""Host-memory pipeline by chunk size and stream count (design tool, GPU box).

    python tools/host_sweep.py [--size 256]

Times cuzfp_hip_compress_host / decompress_host on a pinned 3D f32 array at
rate 8 for each CUZFP_HOST_CHUNK_BYTES x nstreams, beside the bare pinned
H2D / D2H link rates, so the pipeline's defaults can be picked from the
measurement (bench.py reports the default's rates as host_path).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=256)
    p.add_argument("--reps", type=int, default=9)
    a = p.parse_args()
    import torch
    import cuzfp_amd as cz
    from cuzfp_amd.datagen import polynomial_field
    arr = polynomial_field((a.size,) * 3, np.float32)
    mb = cz.rate_to_maxbits(8, np.float32, 3)
    h_in = torch.from_numpy(arr).pin_memory()
    nbytes = cz.stream_bytes(arr.shape, arr.dtype, mb)
    h_s = torch.empty(nbytes // 8, dtype=torch.int64).pin_memory()
    h_out = torch.empty(arr.shape, dtype=torch.float32).pin_memory()
    d = torch.empty_like(h_in, device="cuda")
    ds = torch.empty_like(h_s, device="cuda")

    def rate(fn, n):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        ts.sort()
        return round(n / ts[len(ts) // 2] / 1e9, 2)

    res = {"h2d_GBps": rate(lambda: d.copy_(h_in, non_blocking=True), arr.nbytes),
           "d2h_GBps": rate(lambda: h_s.copy_(ds, non_blocking=True), nbytes), "runs": []}
    print(json.dumps({k: v for k, v in res.items() if k != "runs"}), flush=True)
    s_np = h_s.numpy().view(np.uint64)
    d.copy_(h_in)
    want = cz.decode(cz.encode(d, mb), arr.shape, d.dtype, mb).cpu().numpy().view(np.uint32)
    for zc, ordered, split, chunks in (("0", "0", "1", (8,)), ("0", "1", "0", (32, 64)), ("0", "1", "1", (16, 32, 64)),
                                       ("1", "1", "1", (64,)), ("2", "1", "1", (64,))):
        os.environ["CUZFP_HOST_ZEROCOPY"] = zc
        os.environ["CUZFP_HOST_ORDERED"] = ordered
        os.environ["CUZFP_HOST_SPLIT"] = split
        for chunk_mb in chunks:
            os.environ["CUZFP_HOST_CHUNK_BYTES"] = str(chunk_mb << 20)
            ns = 4
            c = rate(lambda: cz.compress_host(h_in.numpy(), mb, nstreams=ns, out=s_np), arr.nbytes)
            dcp = rate(lambda: cz.decompress_host(s_np, arr.shape, np.float32, mb, nstreams=ns, out=h_out.numpy()),
                       arr.nbytes)
            ok = bool(np.array_equal(h_out.numpy().view(np.uint32), want))
            r = {"zero_copy": zc, "ordered": ordered, "split": split, "chunk_MiB": chunk_mb, "nstreams": ns, "compress_GBps": c,
                 "decompress_GBps": dcp, "roundtrip_equal": ok}
            res["runs"].append(r)
            print(json.dumps(r), flush=True)
    best = max(res["runs"], key=lambda r: r["compress_GBps"] + r["decompress_GBps"])
    print("best", json.dumps(best))


if __name__ == "__main__":
    main()
