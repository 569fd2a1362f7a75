#!/usr/bin/env python3
"""Differential fuzz of the ``cuda_zfp`` CLI against CPU zfp 0.5.0 -- TEST INFRASTRUCTURE.

A Python 3 restatement of the reference's harness ``src/utils/test.py:1-137``: random
array shapes and rates, arrays from ``data_gen``, each compressed by our ``cuda_zfp``
(``cuzfp_amd/bin``, the MI355X codec behind ``libcuZFP.so``) and by the reference's CPU
``zfp`` tool (``oracle/_ref/zfp``, built from zfp-0.5.0/utils/zfp.c by oracle/Makefile);
the two compressed files must be byte-identical, and so must the two decompressed
files (test.py:68-93 runs ``cmp`` on both).

Where this differs from test.py, and why:
* test.py passes ``-t f32`` to CPU ``zfp``, whose 0.5.0 CLI only knows ``-f``/``-d``
  (zfp.c:170-180), and CPU zfp rejects integer fields (zfp.c:618-624): floats go to
  CPU ``zfp`` with ``-f``/``-d``; int32/int64 streams are checked against our oracle
  restatement's integer path (``oracle.restatement``, the block-level
  zfp_encode_block_int32/64 algorithm), the only CPU oracle for them.
* ``--partial`` also draws dims that are not multiples of 4 (CPU zfp's pad_block);
  ``--header`` adds a pass with ``-h`` on both tools (the 96/148-bit zfp header).
* Files go to a temporary directory, not the working directory.

Usage (GPU box):  python tests/fuzz_cli.py [--tests 10] [--seed 0] [--types f32,f64,i32,i64]
                  [--partial] [--header] [--max-dim 400]
Exit status 0 = every case matched.
"""
from __future__ import annotations

import argparse
import os
import random
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "cuzfp_amd", "bin")
CPU_ZFP = os.path.join(ROOT, "oracle", "_ref", "zfp")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
NP_TYPES = {"f32": np.float32, "f64": np.float64, "i32": np.int32, "i64": np.int64}


def dims_args(shape_xyz):
    nx, ny, nz = shape_xyz
    if ny == 0:
        return ["-1", str(nx)]
    if nz == 0:
        return ["-2", str(nx), str(ny)]
    return ["-3", str(nx), str(ny), str(nz)]


def run(cmd, quiet=True):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"{' '.join(cmd)} exited {r.returncode}: {r.stderr.strip()[-400:]}")
    return r


def cpu_maxbits(rate, t, dims):
    """cuZFP's stream_set_rate (zfp_structs.h:61-91) for integer rates: floor(4^d r + .5)."""
    bits = int(np.floor((1 << (2 * dims)) * rate + 0.5))
    if t == "f32":
        bits = max(bits, 9)
    if t == "f64":
        bits = max(bits, 12)
    if dims == 3:
        bits = (bits + 63) & ~63
    return bits


def fuzz_case(tmp, shape_xyz, rate, t, header, log):
    nx, ny, nz = shape_xyz
    dims = 1 + (ny != 0) + (nz != 0)
    dargs = dims_args(shape_xyz)
    raw = os.path.join(tmp, "t_data")
    run([os.path.join(BIN, "data_gen"), "-o", raw, "-t", t] + dargs)
    hdr = ["-h"] if header else []
    ours_z, ours_o = os.path.join(tmp, "t_cmp_ours"), os.path.join(tmp, "t_dec_ours")
    run([os.path.join(BIN, "cuda_zfp"), "-q", "-i", raw, "-t", t, "-r", str(rate), "-z", ours_z] + dargs + hdr)
    if header:
        run([os.path.join(BIN, "cuda_zfp"), "-q", "-h", "-z", ours_z, "-o", ours_o])
    else:
        run([os.path.join(BIN, "cuda_zfp"), "-q", "-z", ours_z, "-t", t, "-r", str(rate), "-o", ours_o] + dargs)
    got_z = open(ours_z, "rb").read()
    got_o = open(ours_o, "rb").read()
    if t in ("f32", "f64"):
        flag = "-f" if t == "f32" else "-d"
        ref_z, ref_o = os.path.join(tmp, "t_cmp_zfp"), os.path.join(tmp, "t_dec_zfp")
        run([CPU_ZFP, "-q", flag, "-i", raw, "-r", str(rate), "-z", ref_z] + dargs + hdr)
        if header:
            run([CPU_ZFP, "-q", "-h", "-z", ref_z, "-o", ref_o])
        else:
            run([CPU_ZFP, "-q", flag, "-z", ref_z, "-r", str(rate), "-o", ref_o] + dargs)
        want_z = open(ref_z, "rb").read()
        want_o = open(ref_o, "rb").read()
    else:
        import oracle
        if oracle.restatement is None:
            oracle.build(with_reference=False)
            oracle.reload()
        shape = tuple(s for s in (nz, ny, nx) if s)
        a = np.fromfile(raw, dtype=NP_TYPES[t]).reshape(shape)
        mb = cpu_maxbits(rate, t, dims)
        want_z = oracle.restatement.compress(a, mb).tobytes()
        want_o = oracle.restatement.decompress(np.frombuffer(want_z, np.uint64), shape, NP_TYPES[t], mb).tobytes()
    ok_z, ok_o = got_z == want_z, got_o == want_o
    log(f"{t} {'x'.join(str(s) for s in shape_xyz if s)} r{rate}{' -h' if header else ''}: "
        f"compressed {'ok' if ok_z else 'DIFFER'} ({len(got_z)} B), decompressed {'ok' if ok_o else 'DIFFER'}")
    return ok_z and ok_o


def draw_shape(rng, dims, partial, max_dim):
    def one():
        if partial:
            return rng.randrange(1, max_dim + 1)
        return rng.randrange(1, max_dim // 4 + 1) * 4  # test.py:103-127: 4*[1,100]
    nx = one()
    ny = one() if dims >= 2 else 0
    nz = one() if dims >= 3 else 0
    return nx, ny, nz


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--tests", type=int, default=10, help="cases per dimensionality (test.py: 10)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--types", default="f32,f64,i32,i64")
    ap.add_argument("--partial", action="store_true", help="also dims that are not multiples of 4")
    ap.add_argument("--header", action="store_true", help="a second pass of every float case with -h")
    ap.add_argument("--max-dim", type=int, default=400, help="largest extent (test.py: 400)")
    ap.add_argument("--max-values", type=int, default=1 << 24, help="redraw shapes above this many values")
    ap.add_argument("--quiet", action="store_true")
    args = ap.parse_args(argv)
    for exe in (os.path.join(BIN, "cuda_zfp"), os.path.join(BIN, "data_gen")):
        if not os.access(exe, os.X_OK):
            print(f"missing {exe}: run `python -c 'import cuzfp_amd.build as b; b.build()'`", file=sys.stderr)
            return 2
    types = args.types.split(",")
    if any(t in ("f32", "f64") for t in types) and not os.access(CPU_ZFP, os.X_OK):
        print(f"missing {CPU_ZFP}: run `make -C oracle ref` where /root/reference exists", file=sys.stderr)
        return 2
    rng = random.Random(args.seed)
    log = (lambda s: None) if args.quiet else (lambda s: print(s, flush=True))
    failures = cases = 0
    with tempfile.TemporaryDirectory(prefix="cuzfp_fuzz_") as tmp:
        for dims in (1, 2, 3):
            for _ in range(args.tests):
                shape = draw_shape(rng, dims, args.partial, args.max_dim)
                while np.prod([s for s in shape if s]) > args.max_values:
                    shape = draw_shape(rng, dims, args.partial, args.max_dim)
                rate = rng.randrange(1, 32)  # test.py:106: rate in [1, 31]
                for t in types:
                    for header in ([False, True] if args.header and t in ("f32", "f64") else [False]):
                        cases += 1
                        if not fuzz_case(tmp, shape, rate, t, header, log):
                            failures += 1
    print(f"fuzz_cli: {cases - failures}/{cases} cases byte-identical", flush=True)
    return 1 if failures else 0


if __name__ == "__main__":
    sys.exit(main())
