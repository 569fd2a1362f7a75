"""Per-SIMD / per-XCD view of the stamped kernels (tools/probe.py stamps output).

    python tools/stamps_simd.py gpurun_out/stamps_encode_polynomial_256.npy [...]

For every SIMD: when its first and last wave started, when its waves' inputs
arrived (encode: end of the gather + exponent phase), when its last wave ended;
then the spread of SIMD end times, by XCD, and how the end time follows the
last input arrival.  Design tool for the launch structure.
"""
from __future__ import annotations

import sys

import numpy as np


def load(path):
    a = np.load(path).astype(np.int64)
    hw, t, rt = a[:, 0], a[:, 1:8], a[:, 8:10]
    r0 = rt[:, 0].min()
    rs, re = (rt[:, 0] - r0) * 10.0, (rt[:, 1] - r0) * 10.0
    rel = (t - t[:, :1]).astype(np.float64)
    xcc = hw >> 32
    simd = (xcc << 16) | (((hw >> 13) & 3) << 12) | (((hw >> 12) & 1) << 11) | (((hw >> 8) & 15) << 4) | ((hw >> 4) & 3)
    cu = simd >> 4
    life = re - rs
    clk = np.median(rel[:, 6] / np.maximum(life, 1))  # memtime cycles per ns
    return dict(rs=rs, re=re, rel=rel, xcc=xcc, simd=simd, cu=cu, clk=clk)


def pct(v, ps=(0, 10, 50, 90, 100)):
    return " ".join(f"{np.percentile(v, p):7.0f}" for p in ps)


def main(paths):
    for path in paths:
        d = load(path)
        enc = "encode" in path
        first_col = 1 if enc else 5  # encode: emax (gather landed); decode: copy-in done
        arrive = d["rs"] + d["rel"][:, first_col] / d["clk"]
        print(f"== {path}: {len(d['rs'])} waves, memtime {d['clk']:.3f} cycles/ns")
        print("   percentiles             min     p10     p50     p90     max  (ns)")
        print("   wave start          ", pct(d["rs"]))
        print("   wave input arrived  ", pct(arrive))
        print("   wave end            ", pct(d["re"]))
        u, inv = np.unique(d["simd"], return_inverse=True)
        s_end = np.full(len(u), -1.0)
        s_last_in = np.full(len(u), -1.0)
        s_first_in = np.full(len(u), 1e18)
        np.maximum.at(s_end, inv, d["re"])
        np.maximum.at(s_last_in, inv, arrive)
        np.minimum.at(s_first_in, inv, arrive)
        s_x = np.zeros(len(u), dtype=np.int64)
        s_x[inv] = d["xcc"]
        print("   SIMD first input    ", pct(s_first_in))
        print("   SIMD last input     ", pct(s_last_in))
        print("   SIMD end            ", pct(s_end))
        busy = s_end - s_first_in
        print("   SIMD end-first_input", pct(busy))
        c = np.corrcoef(s_last_in, s_end)[0, 1]
        c2 = np.corrcoef(s_first_in, s_end)[0, 1]
        print(f"   corr(SIMD end, last input) {c:.2f}   corr(SIMD end, first input) {c2:.2f}")
        for x in np.unique(s_x):
            m = s_x == x
            print(f"   XCD {x}: SIMDs {m.sum():4d}  first input p50 {np.median(s_first_in[m]):7.0f}"
                  f"  last input p50 {np.median(s_last_in[m]):7.0f}  end p10/p50/max "
                  f"{np.percentile(s_end[m], 10):7.0f} {np.median(s_end[m]):7.0f} {s_end[m].max():7.0f}")
        # CU-level: do the 4 SIMDs of a CU end together?
        cu_of = u >> 4
        cu_u, cinv = np.unique(cu_of, return_inverse=True)
        cmax = np.full(len(cu_u), -1.0)
        cmin = np.full(len(cu_u), 1e18)
        np.maximum.at(cmax, cinv, s_end)
        np.minimum.at(cmin, cinv, s_end)
        print("   CU end spread (max-min over its SIMDs)", pct(cmax - cmin))
        print("   CU end                ", pct(cmax))


if __name__ == "__main__":
    main(sys.argv[1:])
