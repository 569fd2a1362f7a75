"""The CPU oracle, pinned before it is trusted (CPU-only).

1. testzfp's own fixtures: fields.c inputs and the polynomial generator match
   testzfp's Jenkins checksums (zfp-0.5.0/tests/testzfp.cpp:475-489).
2. The restatement reproduces every committed golden stream / hash generated
   from the reference's own zfp 0.5.0 (tests/golden/make_golden.py).
3. testzfp's fixed-rate known answers: compressed size == rate * n / 8
   (testzfp.cpp:124-128) and max error <= its table (testzfp.cpp:495-538).
4. When oracle/_ref is built: restatement == reference bit-for-bit on random
   arrays, strides, denormal / tiny blocks and integer blocks.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from cuzfp_amd.datagen import polynomial_field, ramp, splitmix_uniform

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def golden():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)["cases"]


@pytest.fixture(scope="module")
def fields():
    return dict(np.load(os.path.join(GOLDEN, "fields.npz")))


@pytest.fixture(scope="module")
def streams():
    return {k.replace("__", "/"): v for k, v in np.load(os.path.join(GOLDEN, "streams.npz")).items()}


# testzfp.cpp:475-489, TEST_SIZE 4 / 8 / 16
CHECKSUMS = {
    4: {np.float32: [0xdad6fd69, 0x000f8df1, 0x60993f48], np.float64: [0x8d95b1fd, 0x96a0e601, 0x66e77c83]},
    8: {np.float32: [0x269fb420, 0xfc4fd405, 0x733b9643], np.float64: [0x3321e28b, 0xfcb8f0f0, 0xd0f6d6ad]},
    16: {np.float32: [0x62d6c2b5, 0x88aa838e, 0x84f98253], np.float64: [0xf2bd03a4, 0x10084595, 0xb8df0e02]},
}
# testzfp.cpp:495-536 fixed-rate max errors [type][dims-1][rate index]
EMAX = {
    4: {np.float32: [[1.998e+00, 7.767e-03, 0.0], [2.356e-01, 3.939e-04, 7.451e-09], [2.479e-01, 1.525e-03, 7.451e-08]],
        np.float64: [[1.998e+00, 9.976e-01, 1.360e-05], [2.944e+00, 2.491e-02, 2.578e-06], [6.103e-01, 3.253e-02, 6.467e-06]]},
    8: {np.float32: [[2.000e+00, 1.425e-03, 0.0], [7.110e-02, 1.264e-05, 2.329e-10], [1.864e-02, 2.814e-05, 1.193e-07]],
        np.float64: [[2.000e+00, 1.001e+00, 3.084e-06, 0.0], [2.266e+00, 3.509e-03, 1.784e-08, 0.0], [2.494e-01, 1.473e-03, 7.060e-08, 3.470e-18]]},
}
RATES = {np.float32: (2, 8, 32), np.float64: (1, 4, 16, 64)}


def zfp_regression_shape(m, d):
    return {1: (m ** 6,), 2: (m ** 3, m ** 3), 3: (m * m,) * 3}[d]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("d", [1, 2, 3])
def test_fields_checksum(fields, restatement, dtype, d):
    a = fields[f"{'float' if dtype == np.float32 else 'double'}_{d}d"]
    assert restatement.jenkins_hash(a) == CHECKSUMS[4][dtype][d - 1]


@pytest.mark.parametrize("m", [8, 16])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("d", [1, 2, 3])
def test_polynomial_checksum(restatement, m, dtype, d):
    a = polynomial_field(zfp_regression_shape(m, d), dtype)
    assert restatement.jenkins_hash(a) == CHECKSUMS[m][dtype][d - 1]


def test_golden_streams(golden, streams, fields, restatement):
    n = 0
    for name, s in streams.items():
        rec = golden[name]
        if name.startswith("fields/"):
            a = fields[name.split("/")[1]]
        else:
            a = ramp(tuple(rec["shape"]), np.dtype(rec["dtype"]))
        mb = rec["maxbits"]
        got = restatement.compress(a, mb)
        assert np.array_equal(got, s), name
        assert sha(restatement.decompress(s, a.shape, a.dtype, mb)) == rec["decoded_sha256"], name
        n += 1
    assert n >= 27


def test_golden_fuzz(golden, restatement):
    for name, rec in golden.items():
        if not name.startswith("fuzz/"):
            continue
        dt = np.dtype(rec["dtype"])
        a = (splitmix_uniform(tuple(rec["shape"]), dt, rec["seed"]) * (10.0 ** rec["scale_exp10"])).astype(dt)
        s = restatement.compress(a, rec["maxbits"])
        assert sha(s) == rec["stream_sha256"], name
        assert sha(restatement.decompress(s, a.shape, dt, rec["maxbits"])) == rec["decoded_sha256"], name


@pytest.mark.parametrize("name", ["baseline/3d_f32_256_r8/polynomial", "baseline/1d_f32_1M_r8/splitmix",
                                  "baseline/3d_f64_256_r16/polynomial"])
def test_golden_baseline(golden, restatement, name):
    rec = golden[name]
    dt = np.dtype(rec["dtype"])
    shape = tuple(rec["shape"])
    a = polynomial_field(shape, dt) if rec["generator"] == "polynomial" else splitmix_uniform(shape, dt, rec["seed"])
    s = restatement.compress(a, rec["maxbits"])
    assert s.nbytes == rec["bytes"]
    assert sha(s) == rec["stream_sha256"]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("d", [1, 2, 3])
def test_testzfp_fixed_rate_kat(fields, restatement, dtype, d):
    """testzfp.cpp:92-140 test_rate on the TEST_SIZE 4 fields and TEST_SIZE 8 polynomial."""
    for m in (4, 8):
        if m == 4:
            a = fields[f"{'float' if dtype == np.float32 else 'double'}_{d}d"]
        else:
            a = polynomial_field(zfp_regression_shape(8, d), dtype)
        for i, rate in enumerate(RATES[dtype][:len(EMAX[m][dtype][d - 1])]):
            mb = restatement.rate_to_maxbits(rate, dtype, d)
            s = restatement.compress(a, mb)
            actual_rate = mb / 4 ** d  # zfp_stream_set_rate's return value (zfp.c:429)
            assert s.nbytes == int(np.floor(actual_rate * a.size / 8 + 0.5))
            out = restatement.decompress(s, a.shape, dtype, mb)
            err = np.max(np.abs(out.astype(np.float64) - a.astype(np.float64)))
            assert err <= EMAX[m][dtype][d - 1][i], (m, rate, err)


def _rand(rng, shape, dtype, kind):
    if kind == 0:
        a = rng.standard_normal(shape)
    elif kind == 1:
        a = np.cumsum(rng.standard_normal(shape), axis=-1)
    elif kind == 2:
        a = rng.standard_normal(shape) * 10.0 ** rng.integers(-38, 38, size=shape)
    else:
        a = np.where(rng.random(shape) < 0.5, 0, rng.standard_normal(shape))
    with np.errstate(over="ignore"):
        return a.astype(dtype)


@pytest.mark.parametrize("dims", [1, 2, 3])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_restatement_vs_reference(reference, restatement, dims, dtype):
    rng = np.random.default_rng(dims * 10 + (dtype == np.float64))
    for trial in range(25):
        shape = tuple(int(rng.integers(1, 40 if dims < 3 else 14)) for _ in range(dims))
        a = _rand(rng, shape, dtype, trial % 4)
        rate = float(rng.integers(1, 33)) if trial % 3 else float(rng.uniform(0.5, 40))
        mb = reference.rate_to_maxbits(rate, dtype, dims)
        s = reference.compress(a, mb)
        assert np.array_equal(restatement.compress(a, mb), s)
        d1 = reference.decompress(s, shape, dtype, mb)
        d2 = restatement.decompress(s, shape, dtype, mb)
        assert np.array_equal(d1.view(np.uint8), d2.view(np.uint8))


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_restatement_tiny_and_denormal(reference, restatement, dtype):
    """Blocks whose scale factor overflows (x86 cast -> INT_MIN) and denormals."""
    rng = np.random.default_rng(7)
    scales = [1e-30, 1e-38, 1e-44] if dtype == np.float32 else [1e-300, 1e-310, 1e-320]
    for sc in scales:
        for dims in (1, 2, 3):
            a = (rng.standard_normal((8,) * dims) * sc).astype(dtype)
            a.flat[::3] = 0
            for rate in (2, 8, 16, 31):
                mb = reference.rate_to_maxbits(rate, dtype, dims)
                s = reference.compress(a, mb)
                assert np.array_equal(restatement.compress(a, mb), s)
                d1 = reference.decompress(s, a.shape, dtype, mb)
                d2 = restatement.decompress(s, a.shape, dtype, mb)
                assert np.array_equal(d1.view(np.uint8), d2.view(np.uint8))


def test_restatement_strided(reference, restatement):
    """zfp honours strides (compress.c:41-42,70-72); cuZFP ignores them.
    Positive strides only: zfp 0.5.0 mixes `uint mx` with `int sx` in its
    pointer steps (compress.c:232-233, 262-263), so a negative stride wraps
    the pointer and crashes the reference.  Negative strides are exercised
    against the restatement alone (tests/test_gpu_parity.py)."""
    rng = np.random.default_rng(11)
    base = rng.standard_normal((12, 10, 22)).astype(np.float32)
    view = base[::2, :, 1:19]   # z stride of 2 planes, padded x rows
    nz, ny, nx = view.shape
    st = tuple(s // 4 for s in view.strides[::-1])  # (sx, sy, sz) in elements
    mb = 256
    off = (view.__array_interface__["data"][0] - base.__array_interface__["data"][0]) // 4
    import ctypes
    cap = reference.stream_bytes(view.shape, mb) + 64
    out_r = np.zeros(cap // 8, np.uint64)
    out_o = np.zeros(cap // 8, np.uint64)
    ptr = base.ctypes.data + 4 * off
    n1 = reference.lib.ref_compress(3, nx, ny, nz, st[0], st[1], st[2], mb, ptr, out_r.ctypes.data, cap)
    n2 = restatement.lib.oracle_compress(3, nx, ny, nz, st[0], st[1], st[2], mb, ptr, out_o.ctypes.data, cap)
    assert n1 == n2 and np.array_equal(out_r, out_o)
    assert np.array_equal(out_r[: n1 // 8], reference.compress(np.ascontiguousarray(view), mb))
    del ctypes


@pytest.mark.parametrize("dims", [1, 2, 3])
@pytest.mark.parametrize("dtype", [np.int32, np.int64])
def test_restatement_int_blocks(reference, restatement, dims, dtype):
    rng = np.random.default_rng(dims)
    n = 4 ** dims
    nb = 30
    blocks = rng.integers(-2 ** 20, 2 ** 20, size=nb * n).astype(dtype)
    # an array whose raster of blocks is exactly `blocks`: blocks along x only
    shape = {1: (nb * 4,), 2: (4, nb * 4), 3: (4, 4, nb * 4)}[dims]
    B = blocks.reshape((nb,) + (4,) * dims)
    arr = np.concatenate(list(B), axis=dims - 1)
    for mb in (16, 100, 512, 2000):
        s = reference.encode_int_blocks(blocks, dims, mb)
        assert np.array_equal(restatement.compress(arr, mb), s)
        d = restatement.decompress(s, shape, dtype, mb)
        back = np.stack(np.split(d, nb, axis=dims - 1)).reshape(-1)
        assert np.array_equal(back, reference.decode_int_blocks(s, dims, mb, nb, dtype))
