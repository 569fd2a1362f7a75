"""Per-plane event statistics of the 3D fixed-rate encoder (design tool).

Runs zfp's block transform (quantise, lift, reorder, negabinary) vectorised
over every block of a field with numpy, then replays the embedded coder's
control flow per block to count, for each bit plane, how many new ones the
group coder emits before the budget ends.  From those counts it prices the
loop structures a wave64 kernel can use (one block per lane):

  per-plane loop   wave pays  sum_k max_lane(events_k)
  flat loop        wave pays  max_lane sum_k(events_k)

Usage: python tools/plane_stats.py [--field polynomial|splitmix] [--size 256] [--rate 8]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from cuzfp_amd import datagen  # noqa: E402

_P3 = []
for s in [(0,0,0),(1,0,0),(0,1,0),(0,0,1),(0,1,1),(1,0,1),(1,1,0),(2,0,0),(0,2,0),(0,0,2),(1,1,1),
          (2,1,0),(2,0,1),(0,2,1),(1,2,0),(1,0,2),(0,1,2),(3,0,0),(0,3,0),(0,0,3),(2,1,1),(1,2,1),
          (1,1,2),(0,2,2),(2,0,2),(2,2,0),(3,1,0),(3,0,1),(0,3,1),(1,3,0),(1,0,3),(0,1,3),(1,2,2),
          (2,1,2),(2,2,1),(3,1,1),(1,3,1),(1,1,3),(3,2,0),(3,0,2),(0,3,2),(2,3,0),(2,0,3),(0,2,3),
          (2,2,2),(3,2,1),(3,1,2),(1,3,2),(2,3,1),(2,1,3),(1,2,3),(0,3,3),(3,0,3),(3,3,0),(3,2,2),
          (2,3,2),(2,2,3),(1,3,3),(3,1,3),(3,3,1),(2,3,3),(3,2,3),(3,3,2),(3,3,3)]:
    _P3.append(s[0] + 4 * (s[1] + 4 * s[2]))


def _lift(a, axis):
    x, y, z, w = (np.take(a, i, axis=axis).copy() for i in range(4))
    x += w; x >>= 1; w -= x
    z += y; z >>= 1; y -= z
    x += z; x >>= 1; z -= x
    w += y; w >>= 1; y -= w
    w += y >> 1; y -= w >> 1
    return np.stack([x, y, z, w], axis=axis)


def block_coeffs(f):
    nz, ny, nx = f.shape
    b = f.reshape(nz // 4, 4, ny // 4, 4, nx // 4, 4).transpose(0, 2, 4, 1, 3, 5).reshape(-1, 4, 4, 4)
    m = np.abs(b.astype(np.float64)).reshape(len(b), -1).max(axis=1)
    _, e = np.frexp(m)
    e = np.where(m > 0, e, -127)
    q = np.ldexp(b.astype(np.float64), (30 - e)[:, None, None, None]).astype(np.int64).astype(np.int32)
    q = q.astype(np.int32)
    # axes: (block, z, y, x); lift x, then y, then z
    q = _lift(q, 3)
    q = _lift(q, 2)
    q = _lift(q, 1)
    q = q.reshape(len(b), 64)[:, _P3].astype(np.uint32)
    u = (q + np.uint32(0xAAAAAAAA)) ^ np.uint32(0xAAAAAAAA)
    return u


def events(u, budget):
    """ones[b, k]: new ones emitted in plane k; active[b, k]: plane coded at all."""
    nb = len(u)
    bits_le = ((u[:, :, None] >> np.arange(32, dtype=np.uint32)[None, None, :]) & 1).astype(np.uint8)
    ones = np.zeros((nb, 32), np.int32)
    active = np.zeros((nb, 32), bool)
    n = np.zeros(nb, np.int64)
    bits = np.full(nb, budget, np.int64)
    for kk, k in enumerate(range(31, -1, -1)):
        plane = bits_le[:, :, k]
        act = bits > 0
        active[:, kk] = act
        bits -= np.minimum(n, bits)
        # highest one at position >= n
        pos = np.arange(64)[None, :]
        newmask = (plane == 1) & (pos >= n[:, None])
        cnt = newmask.sum(1)
        hi = np.where(newmask.any(1), 63 - np.argmax(newmask[:, ::-1], axis=1), -1)
        cost = np.where(cnt > 0, 1 + (hi + 1 - n) + cnt - np.where(hi == 63, 2, 0), np.where(n < 64, 1, 0))
        ones[:, kk] = np.where(act, cnt, 0)
        bits = np.maximum(bits - cost, 0)
        n = np.where(act & (cnt > 0), np.maximum(n, hi + 1), n)
    return ones, active


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--field", default="polynomial")
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--rate", type=float, default=8)
    a = ap.parse_args()
    s = a.size
    if a.field == "polynomial":
        f = datagen.polynomial_field((s, s, s))
    else:
        f = datagen.splitmix_uniform(s ** 3).reshape(s, s, s).astype(np.float32)
    u = block_coeffs(f)
    budget = int(a.rate * 64) - 9
    ones, active = events(u, budget)
    nb = len(u)
    w = nb // 64
    ev = ones + active  # one trip per new one + one per coded plane
    o = ones.reshape(w, 64, 32)
    e = ev.reshape(w, 64, 32)
    act = active.reshape(w, 64, 32)
    print(f"blocks {nb}  planes coded/lane {active.sum(1).mean():.2f}  wave planes {act.any(1).sum(1).mean():.2f}")
    print(f"new ones/lane {ones.sum(1).mean():.2f}  max ones/plane/lane {ones.max(1).mean():.2f}")
    print(f"per-plane loop: wave one-trips {o.max(1).sum(1).mean():.2f}  (lane avg {ones.sum(1).mean():.2f})")
    print(f"flat loop:      wave events {e.sum(2).max(1).mean():.2f}  (lane avg {ev.sum(1).mean():.2f})")
    for per in (2, 4):
        t = (o + per - 1) // per
        print(f"{per} ones/trip: wave trips {t.max(1).sum(1).mean():.2f}")
    hist = np.bincount(o.max(1).ravel(), minlength=20)
    print("hist of per-plane wave max ones:", hist[:20])
    print("mean wave max ones by plane:", np.round(o.max(1).mean(0), 2))


if __name__ == "__main__":
    main()
