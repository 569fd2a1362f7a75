"""Generate tests/golden/ from the reference's own CPU zfp 0.5.0 -- TEST INFRASTRUCTURE.

Run in the build container (it needs /root/reference and oracle/_ref):

    python tests/golden/make_golden.py

Outputs (all data, no reference source):
  fields.npz   the testzfp regression inputs (zfp-0.5.0/tests/fields.c, C99
               hex-float branch) decoded to float32/float64 arrays:
               float_{1,2,3}d, double_{1,2,3}d -- pinned by testzfp's Jenkins
               checksums (testzfp.cpp:475-489).
  streams.npz  reference compressed streams of those fields at testzfp's
               fixed rates (f32: 2, 8, 32; f64: 1, 4, 16, 64 -- testzfp.cpp:491-538)
               and of the sanity ramps of src/tests/t_sanity_check_{1,2,3}.cpp.
  golden.json  per case: shape, dtype, maxbits, compressed bytes, SHA-256 of the
               reference stream and of its decompressed array, max abs error;
               plus the same for seeded splitmix64 fuzz cases (the dims/rate space
               of src/utils/test.py:101-132) and for BASELINE.json's full-size
               configurations (hashes only), including configs[4]'s 1024^3
               array with the word-range hashes of its z-slab shards.
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from cuzfp_amd.datagen import polynomial_field, ramp, splitmix_uniform  # noqa: E402

FIELDS_C = "/root/reference/src/thirdparty_builtin/zfp-0.5.0/tests/fields.c"
SHAPES = {1: (4096,), 2: (64, 64), 3: (16, 16, 16)}


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def parse_fields() -> dict:
    """Decode the C99 hex-float branch of fields.c into numpy arrays."""
    text = open(FIELDS_C).read()
    out = {}
    for name, dt in (("array_float", np.float32), ("array_double", np.float64)):
        start = text.index(name)
        body = text[start:]
        c99 = body[body.index("#if"):body.index("#else")]
        groups = c99.split("},{")
        assert len(groups) == 3, name
        for d, g in enumerate(groups, start=1):
            vals = [float.fromhex(t) for t in re.findall(r"-?0x[0-9a-fA-F.]+p[-+]?\d+", g)]
            assert len(vals) == 4096, (name, d, len(vals))
            out[f"{'float' if dt == np.float32 else 'double'}_{d}d"] = (
                np.array(vals, dtype=dt).reshape(SHAPES[d]))
    return out


def case(ref, a: np.ndarray, maxbits: int, keep_stream: bool):
    s = ref.compress(a, maxbits)
    d = ref.decompress(s, a.shape, a.dtype, maxbits)
    err = float(np.max(np.abs(d.astype(np.float64) - a.astype(np.float64)))) if a.size else 0.0
    rec = {"shape": list(a.shape), "dtype": a.dtype.name, "maxbits": int(maxbits),
           "bytes": int(s.nbytes), "stream_sha256": sha(s), "decoded_sha256": sha(d),
           "max_abs_err": err}
    return rec, (s if keep_stream else None)


def add_sharded_1024(golden: dict, ref) -> None:
    """BASELINE configs[4]: the 1024^3 f32 polynomial field at rate 8, the array
    the bench shards over N GPUs as z-slabs of 1024/N planes.  Hashes of the
    whole stream, of its N equal word ranges (N = 2, 4, 8: rank r's slab
    encodes to words [r*W/N, (r+1)*W/N)) and of the decoded array."""
    shape, dt, rate = (1024, 1024, 1024), np.float32, 8
    a = polynomial_field(shape, dt)
    mb = ref.rate_to_maxbits(rate, dt, 3)
    s = ref.compress(a, mb)
    d = ref.decompress(s, shape, dt, mb)
    rec = {"shape": list(shape), "dtype": "float32", "maxbits": int(mb), "bytes": int(s.nbytes),
           "stream_sha256": sha(s), "decoded_sha256": sha(d), "rate": rate, "generator": "polynomial",
           "max_abs_err": float(np.max(np.abs(d.astype(np.float64) - a.astype(np.float64))))}
    for n in (2, 4, 8):
        w = s.size // n
        rec[f"slab_sha256_n{n}"] = [sha(s[r * w:(r + 1) * w]) for r in range(n)]
    golden["cases"]["baseline/3d_f32_1024_r8/polynomial"] = rec
    print("baseline/3d_f32_1024_r8", rec["bytes"], rec["max_abs_err"], flush=True)


def main() -> None:
    if "--only-1024" in sys.argv:  # append configs[4] to an existing golden.json
        oracle.build(with_reference=True)
        oracle.reload()
        path = os.path.join(HERE, "golden.json")
        golden = json.load(open(path))
        add_sharded_1024(golden, oracle.reference)
        with open(path, "w") as f:
            json.dump(golden, f, indent=1, sort_keys=True)
        return
    oracle.build(with_reference=True)
    oracle.reload()
    ref = oracle.reference
    assert ref is not None, "oracle/_ref not built"
    golden = {"generator": "tests/golden/make_golden.py", "reference": "zfp 0.5.0 (mclarsen/cuZFP "
              "src/thirdparty_builtin/zfp-0.5.0) via oracle/_ref/libzfp_ref.so", "cases": {}}
    streams = {}

    # 1. testzfp fields at testzfp's fixed rates
    fields = parse_fields()
    np.savez_compressed(os.path.join(HERE, "fields.npz"), **fields)
    for key, a in fields.items():
        d = a.ndim
        rates = (2, 8, 32) if a.dtype == np.float32 else (1, 4, 16, 64)
        for rate in rates:
            mb = ref.rate_to_maxbits(rate, a.dtype, d)
            name = f"fields/{key}/r{rate}"
            rec, s = case(ref, a, mb, True)
            rec["rate"] = rate
            golden["cases"][name] = rec
            streams[name] = s

    # 2. sanity ramps (t_sanity_check_{1,2,3}.cpp: rate 8; 3D via cuZFP's
    #    stream_set_rate, which rounds 3D up to a multiple of 64 bits)
    for d, shape in ((1, (128,)), (2, (4, 4)), (3, (4, 8, 16))):
        for dt in (np.float32, np.float64):
            a = ramp(shape, dt)
            mb = ref.rate_to_maxbits(8, dt, d, wra=(d == 3))
            name = f"ramp/{d}d/{np.dtype(dt).name}"
            rec, s = case(ref, a, mb, True)
            golden["cases"][name] = rec
            streams[name] = s

    # 3. seeded fuzz (test.py:101-132 space: dims random, rate 1..31, f32/f64)
    rng = np.random.default_rng(20240601)
    for i in range(48):
        d = 1 + i % 3
        dt = np.float32 if (i // 3) % 2 == 0 else np.float64
        hi = {1: 400, 2: 100, 3: 40}[d]
        shape = tuple(int(rng.integers(1, hi + 1)) for _ in range(d))
        rate = int(rng.integers(1, 32))
        seed = 1000 + i
        a = splitmix_uniform(shape, dt, seed=seed) * (10.0 ** (i % 7 - 3))
        a = a.astype(dt)
        mb = ref.rate_to_maxbits(rate, dt, d)
        rec, _ = case(ref, a, mb, False)
        rec.update({"rate": rate, "seed": seed, "scale_exp10": i % 7 - 3, "generator": "splitmix"})
        golden["cases"][f"fuzz/{i:02d}"] = rec

    # 4. BASELINE.json configurations (hashes only)
    big = [("baseline/3d_f32_256_r8", (256, 256, 256), np.float32, 8),
           ("baseline/3d_f64_256_r16", (256, 256, 256), np.float64, 16),
           ("baseline/2d_f32_8192_r2", (8192, 8192), np.float32, 2),
           ("baseline/1d_f32_1M_r8", (1 << 20,), np.float32, 8)]
    for name, shape, dt, rate in big:
        for gen in ("polynomial", "splitmix"):
            a = polynomial_field(shape, dt) if gen == "polynomial" else splitmix_uniform(shape, dt, 42)
            mb = ref.rate_to_maxbits(rate, dt, len(shape))
            rec, _ = case(ref, a, mb, False)
            rec.update({"rate": rate, "generator": gen, "seed": 42})
            golden["cases"][f"{name}/{gen}"] = rec
            print(name, gen, rec["bytes"], rec["max_abs_err"], flush=True)

    add_sharded_1024(golden, ref)

    np.savez_compressed(os.path.join(HERE, "streams.npz"), **{k.replace("/", "__"): v
                                                               for k, v in streams.items()})
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(golden, f, indent=1, sort_keys=True)
    print("wrote", len(golden["cases"]), "cases")


if __name__ == "__main__":
    main()
