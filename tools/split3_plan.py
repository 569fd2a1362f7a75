"""Search the lane-pair layout of the split 3D encoder (cuzfp_amd/csrc/split3.hpp).

A block is split over lanes A (l) and B (l + 32).  A gathers z = 0, 1 and B
z = 2, 3 (register zl*16 + y*4 + x).  After the x and y lifts, one
v_permlane32_swap per register pair (zl, c) <-> (zl, pi(c)), c in K, hands A
the columns K and B their partners pi(K) for the z lifts.  Then A must hold the
coefficients perm[0..31] and B perm[32..63] (the two 32-bit halves of every
bit plane), in registers that pair perm[t] (A) with perm[32+t] (B): movers go
across with one swap each, and every transpose input whose two halves sit in
different registers costs one select.  This script picks K, pi and the mover
pairing with the fewest selects and prints the tables split3.hpp embeds.
"""
import itertools
import random

PERM = [(0,0,0),(1,0,0),(0,1,0),(0,0,1),(0,1,1),(1,0,1),(1,1,0),(2,0,0),(0,2,0),(0,0,2),(1,1,1),(2,1,0),(2,0,1),
        (0,2,1),(1,2,0),(1,0,2),(0,1,2),(3,0,0),(0,3,0),(0,0,3),(2,1,1),(1,2,1),(1,1,2),(0,2,2),(2,0,2),(2,2,0),
        (3,1,0),(3,0,1),(0,3,1),(1,3,0),(1,0,3),(0,1,3),(1,2,2),(2,1,2),(2,2,1),(3,1,1),(1,3,1),(1,1,3),(3,2,0),
        (3,0,2),(0,3,2),(2,3,0),(2,0,3),(0,2,3),(2,2,2),(3,2,1),(3,1,2),(1,3,2),(2,3,1),(2,1,3),(1,2,3),(0,3,3),
        (3,0,3),(3,3,0),(3,2,2),(2,3,2),(2,2,3),(1,3,3),(3,1,3),(3,3,1),(2,3,3),(3,2,3),(3,3,2),(3,3,3)]
P = [x + 4 * y + 16 * z for (x, y, z) in PERM]
A_SET = set(P[:32])


def contents(K, pi):
    """(A, B) coefficient of every register after the z exchange."""
    A, B = [None] * 32, [None] * 32
    inv = {pi[c]: c for c in K}
    for zl in range(2):
        for cc in range(16):
            r = zl * 16 + cc
            if cc in K:
                A[r] = cc + 16 * zl
                B[r] = pi[cc] + 16 * zl
            else:
                A[r] = inv[cc] + 16 * (2 + zl)
                B[r] = cc + 16 * (2 + zl)
    return A, B


def plan(K, pi, rng=None, tries=1):
    A, B = contents(K, pi)
    a_out = [r for r in range(32) if A[r] not in A_SET]      # A-half must go to B
    b_in = [r for r in range(32) if B[r] in A_SET]           # B-half must go to A
    assert len(a_out) == len(b_in)
    if set(a_out) & set(b_in):  # a register whose both halves must cross: not one swap
        return None
    best = None
    perms = [b_in] if rng is None else [rng.sample(b_in, len(b_in)) for _ in range(tries)]
    for bo in perms:
        A2, B2 = A[:], B[:]
        swaps = []
        for v1, v0 in zip(a_out, bo):      # swap(v0, v1): v0 = (a0, a1), v1 = (b0, b1)
            a0, b0, a1, b1 = A2[v0], B2[v0], A2[v1], B2[v1]
            A2[v0], B2[v0], A2[v1], B2[v1] = a0, a1, b0, b1
            swaps.append((v0, v1))
        whereA = {A2[r]: r for r in range(32)}
        whereB = {B2[r]: r for r in range(32)}
        src = [(whereA[P[t]], whereB[P[32 + t]]) for t in range(32)]
        sel = sum(1 for a, b in src if a != b)
        if best is None or sel < best[0]:
            best = (sel, swaps, src)
    return best


def search(seed=1, iters=20000):
    rng = random.Random(seed)
    cols = list(range(16))
    s = lambda c: (c & 3) + (c >> 2)
    best = None
    for it in range(iters):
        if it == 0:
            K = sorted(cols, key=lambda c: (s(c), c))[:8]
        else:
            K = sorted(rng.sample(cols, 8))
        rest = [c for c in cols if c not in K]
        rng.shuffle(rest)
        pi = dict(zip(K, rest))
        got = plan(K, pi, rng, 8)
        if got is None:
            continue
        sel, swaps, src = got
        key = (sel, len(swaps))
        if best is None or key < best[0]:
            best = (key, K, pi, swaps, src)
    return best


if __name__ == "__main__":
    (sel, nsw), K, pi, swaps, src = search()
    print(f"selects {sel}, mover swaps {nsw}")
    print("K", K)
    print("pi", [pi[c] for c in K])
    print("swaps", swaps)
    print("srcA", [a for a, b in src])
    print("srcB", [b for a, b in src])
