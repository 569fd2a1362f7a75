"""Where the encode+decode step spends the time the two kernels alone do not
(design tool, GPU box): hipGraph-replayed sequences of the 3D f32 256^3 rate-8
kernels, microseconds per launch or per pair.

  python tools/step_gap.py [--size S]

  E / D        encode (decode) back to back, the same buffers
  ED           the bench step: encode x -> w, decode w -> y
  ED'          encode x -> w, decode a second stream w2 -> y (decode input not
               just written)
  E D2         encode x -> w, decode w -> y2 (a second output buffer)
  E c D        the step with a 4-byte copy kernel between the two
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
    a = ap.parse_args()
    import torch
    import cuzfp_amd as cz
    from cuzfp_amd.datagen import polynomial_field
    shape = (a.size,) * 3
    x = torch.from_numpy(polynomial_field(shape)).cuda()
    mb = cz.rate_to_maxbits(8, x.cpu().numpy().dtype, 3)
    w = cz.encode(x, mb)
    w2 = w.clone()
    y = cz.decode(w, shape, x.dtype, mb)
    y2 = torch.empty_like(y)
    s4 = torch.zeros(1024, device="cuda")
    d4 = torch.zeros(1024, device="cuda")
    E = lambda: cz.encode(x, mb, out=w)
    D = lambda: cz.decode(w, shape, x.dtype, mb, out=y)
    seqs = {
        "E": [E],
        "D": [D],
        "ED": [E, D],
        "ED'": [E, lambda: cz.decode(w2, shape, x.dtype, mb, out=y)],
        "E D2": [E, lambda: cz.decode(w, shape, x.dtype, mb, out=y2)],
        "E c D": [E, lambda: cz.copy(s4, d4), D],
        "c": [lambda: cz.copy(s4, d4)],
    }
    res = {}
    for name, fns in seqs.items():
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(10):
                for f in fns:
                    f()
        g.replay()
        torch.cuda.synchronize()
        r = []
        for _ in range(9):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(4):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            r.append(e0.elapsed_time(e1) / 40 * 1000)
        res[name] = round(sorted(r)[4], 2)
        print(f"{name:8s} {res[name]:8.2f} us", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
