"""GPU parity: the HIP codec (through the C-ABI) against the CPU oracle.

Bar: compressed streams bit-exact with zfp 0.5.0 fixed-rate
mode, decompressed arrays bit-exact with zfp 0.5.0's decoder.  Cases follow the
reference's own tests -- the sanity ramps (src/tests/t_sanity_check_{1,2,3}.cpp),
the differential fuzz space of src/utils/test.py:101-132 (random dims, rates
1..31, f32/f64) -- plus partial blocks, strides, integer fields and
denormal / zero / huge-range blocks.
"""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import cuzfp_amd as cz


def _to_dev(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _gpu_roundtrip(a, maxbits, dev):
    import torch
    x = _to_dev(a, dev)
    words = cz.encode(x, maxbits)
    y = cz.decode(words, a.shape, x.dtype, maxbits)
    torch.cuda.synchronize()
    return words.cpu().numpy().view(np.uint64), y.cpu().numpy()


def _fields(rng, shape, dtype, kind):
    if kind == "normal":
        a = rng.standard_normal(shape)
    elif kind == "smooth":
        a = np.cumsum(rng.standard_normal(shape), axis=-1)
    elif kind == "range":
        a = rng.standard_normal(shape) * 10.0 ** rng.integers(-30, 30, size=shape)
    elif kind == "sparse":
        a = np.where(rng.random(shape) < 0.6, 0.0, rng.standard_normal(shape))
    else:
        raise ValueError(kind)
    with np.errstate(over="ignore"):
        return a.astype(dtype)


@pytest.mark.parametrize("dims", [1, 2, 3])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_sanity_ramp(dims, dtype, cuda, restatement):
    # t_sanity_check_{1,2,3}.cpp: f[i] = i at rate 8 round-trips to integers
    shape = {1: (128,), 2: (4, 4), 3: (4, 8, 16)}[dims]
    a = np.arange(np.prod(shape), dtype=dtype).reshape(shape)
    mb = cz.rate_to_maxbits(8, dtype, dims, wra=dims == 3)
    words, y = _gpu_roundtrip(a, mb, cuda)
    ref = restatement.compress(a, mb)
    assert np.array_equal(words, ref)
    assert np.array_equal(y, restatement.decompress(ref, shape, dtype, mb))
    if dtype == np.float32:  # the reference's assertion (f32 only there)
        assert np.array_equal(y.astype(np.int64), a.astype(np.int64))


@pytest.mark.parametrize("dims", [1, 2, 3])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("kind", ["normal", "smooth", "range", "sparse"])
def test_fuzz_vs_oracle(dims, dtype, kind, cuda, restatement):
    # (a stable seed: hash() of a str is salted per process by PYTHONHASHSEED)
    rng = np.random.default_rng(zlib.crc32(f"{dims}/{np.dtype(dtype).str}/{kind}".encode()))
    for trial in range(6):
        hi = {1: 400, 2: 100, 3: 24}[dims]
        shape = tuple(int(rng.integers(1, hi)) for _ in range(dims))
        rate = int(rng.integers(1, 32)) if trial % 2 else float(rng.uniform(0.3, 40))
        mb = cz.rate_to_maxbits(rate, dtype, dims)
        a = _fields(rng, shape, dtype, kind)
        words, y = _gpu_roundtrip(a, mb, cuda)
        ref = restatement.compress(a, mb)
        assert np.array_equal(words, ref), (shape, mb)
        dref = restatement.decompress(ref, shape, dtype, mb)
        assert np.array_equal(y.view(np.uint8), dref.view(np.uint8)), (shape, mb)


# --------------------------------------------------------------------------
# committed golden fixtures (reference zfp 0.5.0 output, tests/golden/)

import hashlib
import json
import os

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _golden():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)["cases"]


def test_golden_fields_and_ramps(cuda):
    from cuzfp_amd.datagen import ramp
    g = _golden()
    fields = dict(np.load(os.path.join(GOLDEN, "fields.npz")))
    streams = {k.replace("__", "/"): v for k, v in np.load(os.path.join(GOLDEN, "streams.npz")).items()}
    for name, s in streams.items():
        rec = g[name]
        a = fields[name.split("/")[1]] if name.startswith("fields/") else ramp(tuple(rec["shape"]), np.dtype(rec["dtype"]))
        words, y = _gpu_roundtrip(a, rec["maxbits"], cuda)
        assert np.array_equal(words, s), name
        # decoding the reference stream reproduces the reference's decoded array
        import torch
        dec = cz.decode(torch.from_numpy(s.view(np.int64).copy()).to(cuda), a.shape,
                        torch.from_numpy(a).dtype, rec["maxbits"]).cpu().numpy()
        assert _sha(dec) == rec["decoded_sha256"], name


def test_golden_fuzz(cuda):
    from cuzfp_amd.datagen import splitmix_uniform
    for name, rec in _golden().items():
        if not name.startswith("fuzz/"):
            continue
        dt = np.dtype(rec["dtype"])
        a = (splitmix_uniform(tuple(rec["shape"]), dt, rec["seed"]) * (10.0 ** rec["scale_exp10"])).astype(dt)
        words, y = _gpu_roundtrip(a, rec["maxbits"], cuda)
        assert _sha(words) == rec["stream_sha256"], name
        assert _sha(y) == rec["decoded_sha256"], name


@pytest.mark.parametrize("name", ["baseline/3d_f32_256_r8", "baseline/3d_f64_256_r16",
                                  "baseline/2d_f32_8192_r2", "baseline/1d_f32_1M_r8"])
@pytest.mark.parametrize("gen", ["polynomial", "splitmix"])
def test_golden_baseline_configs(cuda, name, gen):
    """BASELINE.json's full-size configurations: stream and decoded array hash-equal
    to the reference's own zfp 0.5.0 output."""
    from cuzfp_amd.datagen import polynomial_field, splitmix_uniform
    rec = _golden()[f"{name}/{gen}"]
    dt = np.dtype(rec["dtype"])
    shape = tuple(rec["shape"])
    a = polynomial_field(shape, dt) if gen == "polynomial" else splitmix_uniform(shape, dt, rec["seed"])
    words, y = _gpu_roundtrip(a, rec["maxbits"], cuda)
    assert words.nbytes == rec["bytes"]
    assert _sha(words) == rec["stream_sha256"]
    assert _sha(y) == rec["decoded_sha256"]


# --------------------------------------------------------------------------
# integer fields, strides, extremes, host pipeline, sizes


@pytest.mark.parametrize("dims", [1, 2, 3])
@pytest.mark.parametrize("dtype", [np.int32, np.int64])
def test_int_fields(cuda, restatement, dims, dtype):
    rng = np.random.default_rng(dims * 3 + (dtype == np.int64))
    for trial in range(6):
        hi = {1: 300, 2: 60, 3: 20}[dims]
        shape = tuple(int(rng.integers(1, hi)) for _ in range(dims))
        lim = 2 ** (20 if trial % 2 else 30)
        a = rng.integers(-lim, lim, size=shape).astype(dtype)
        mb = int(rng.integers(2, 3000))
        words, y = _gpu_roundtrip(a, mb, cuda)
        ref = restatement.compress(a, mb)
        assert np.array_equal(words, ref)
        assert np.array_equal(y, restatement.decompress(ref, shape, dtype, mb))


def test_strided_views(cuda, restatement):
    """Non-contiguous device views vs the restatement with the same strides (zfp
    honours sx/sy/sz; cuZFP ignored them).  torch views give positive strides;
    negative strides go through the C-ABI with a hand-made base pointer."""
    import ctypes
    import torch
    rng = np.random.default_rng(21)
    base = rng.standard_normal((16, 12, 26)).astype(np.float32)
    tb = torch.from_numpy(base).to(cuda)
    mb = 384
    cases = [((slice(None, None, 2), slice(None), slice(1, 19)), None),
             ((slice(3, 14), slice(2, 11), slice(None, None, 3)), None),
             ((slice(None), slice(None, None, -1), slice(None, None, -2)), "negative")]
    lib = cz.library()
    for sl, kind in cases:
        view_n = base[sl]
        nz, ny, nx = view_n.shape
        st = tuple(s // 4 for s in view_n.strides[::-1])
        off = (view_n.__array_interface__["data"][0] - base.__array_interface__["data"][0]) // 4
        cap = restatement.stream_bytes(view_n.shape, mb) + 64
        ref = np.zeros(cap // 8, np.uint64)
        n = restatement.lib.oracle_compress(3, nx, ny, nz, st[0], st[1], st[2], mb,
                                            view_n.__array_interface__["data"][0], ref.ctypes.data, cap)
        ref = ref[: n // 8]
        if kind is None:
            words = cz.encode(tb[sl], mb)
        else:
            words = torch.empty(n // 8, dtype=torch.int64, device=cuda)
            got = ctypes.c_size_t(0)
            rc = lib.cuzfp_hip_encode(tb.data_ptr() + 4 * off, 3, nx, ny, nz, st[0], st[1], st[2], mb,
                                      words.data_ptr(), n, ctypes.byref(got), None)
            assert rc == 0
        torch.cuda.synchronize()
        assert np.array_equal(words.cpu().numpy().view(np.uint64), ref), kind
        # decode into a strided destination, leaving the gaps untouched
        dst = torch.full_like(tb, -7.0)
        rc = lib.cuzfp_hip_decode(words.data_ptr(), n, 3, nx, ny, nz, st[0], st[1], st[2], mb,
                                  dst.data_ptr() + 4 * off, None)
        assert rc == 0
        torch.cuda.synchronize()
        got = dst.cpu().numpy()
        want = restatement.decompress(ref, view_n.shape, np.float32, mb)
        assert np.array_equal(got[sl], want)
        mask = np.ones(base.shape, bool)
        mask[sl] = False
        assert np.all(got[mask] == -7.0)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_extreme_blocks(cuda, restatement, dtype):
    rng = np.random.default_rng(9)
    scales = [1e-30, 1e-38, 1e-44, 3e38] if dtype == np.float32 else [1e-300, 1e-310, 1e-320, 1e308]
    for sc in scales:
        a = (rng.standard_normal((12, 8, 8)) * sc).astype(dtype)
        a.flat[::5] = 0
        a[0, 0, 0] = np.inf if sc > 1 else a[0, 0, 0]
        a[6, 4, 4] = np.nan if sc > 1 else a[6, 4, 4]  # a NaN in another block
        for mb in (restatement.rate_to_maxbits(1, dtype, 3), 512, 1000, 4171):
            words, y = _gpu_roundtrip(a, mb, cuda)
            ref = restatement.compress(a, mb)
            assert np.array_equal(words, ref)
            assert np.array_equal(y.view(np.uint8), restatement.decompress(ref, a.shape, dtype, mb).view(np.uint8))


@pytest.mark.parametrize("shape", [(1,), (3,), (5, 7), (1, 1, 1), (2, 3, 5), (64, 64, 64), (4, 4, 4 * 4097)])
def test_edge_sizes(cuda, restatement, shape):
    """Empty-ish, ragged and multi-wave arrays (a wave = 64 blocks)."""
    from cuzfp_amd.datagen import splitmix_uniform
    for mb in (9, 32, 77, 512):
        a = splitmix_uniform(shape, np.float32, seed=len(shape) + mb)
        words, y = _gpu_roundtrip(a, mb, cuda)
        ref = restatement.compress(a, mb)
        assert np.array_equal(words, ref), (shape, mb)
        assert np.array_equal(y, restatement.decompress(ref, shape, np.float32, mb))


@pytest.mark.parametrize("shape,dtype,rate", [((96, 80, 72), np.float32, 8), ((40, 36, 20), np.float64, 16),
                                              ((1000, 700), np.float32, 2), ((300001,), np.float32, 8),
                                              ((33, 34, 35), np.float32, 5.5)])
@pytest.mark.parametrize("pinned", [False, True])
def test_host_pipeline(cuda, restatement, shape, dtype, rate, pinned):
    """cuzfp_hip_compress_host / decompress_host (pinned chunked pipeline) ==
    the device path == the oracle, from pageable and from pinned buffers."""
    import torch
    from cuzfp_amd.datagen import splitmix_uniform
    a = splitmix_uniform(shape, dtype, seed=5)
    mb = cz.rate_to_maxbits(rate, dtype, len(shape))
    out = None
    if pinned:
        host = torch.from_numpy(a).pin_memory()
        a = host.numpy()
        out = torch.empty(cz.stream_bytes(shape, dtype, mb) // 8, dtype=torch.int64).pin_memory().numpy().view(np.uint64)
    for nstreams in (1, 3):
        s = cz.compress_host(a, mb, nstreams=nstreams, out=out)
        ref = restatement.compress(a, mb)
        assert np.array_equal(s, ref)
        y = cz.decompress_host(s, shape, dtype, mb, nstreams=nstreams)
        assert np.array_equal(y, restatement.decompress(ref, shape, dtype, mb))


@pytest.mark.gpu
@pytest.mark.parametrize("zero_copy", ["1", "2"])
def test_host_zero_copy_views(cuda, restatement, monkeypatch, zero_copy):
    """Zero-copy host paths on pinned buffers that are views inside larger
    pinned allocations (offset starts, a stream buffer larger than the stream):
    byte-equal to the oracle, and the bytes around the views untouched."""
    import torch
    from cuzfp_amd.datagen import splitmix_uniform
    monkeypatch.setenv("CUZFP_HOST_ZEROCOPY", zero_copy)
    shape, dtype, mb = (40, 36, 28), np.float32, cz.rate_to_maxbits(8, np.float32, 3)
    a = splitmix_uniform(shape, dtype, seed=11)
    n = a.size
    big = torch.zeros(n + 64, dtype=torch.float32).pin_memory().numpy()
    big[16:16 + n] = a.ravel()
    view = big[16:16 + n].reshape(shape)
    nw = cz.stream_bytes(shape, dtype, mb) // 8
    sbig = torch.full((nw + 40,), -1, dtype=torch.int64).pin_memory().numpy().view(np.uint64)
    sview = sbig[8:8 + nw + 16]  # capacity beyond the stream
    ref = restatement.compress(a, mb)
    want = restatement.decompress(ref, shape, dtype, mb)
    s = cz.compress_host(view, mb, out=sview)[:nw]
    assert np.array_equal(s, ref)
    assert np.all(sbig[:8] == np.uint64(2**64 - 1)) and np.all(sbig[8 + nw:] == np.uint64(2**64 - 1))
    ybig = torch.full((n + 64,), 7.0, dtype=torch.float32).pin_memory().numpy()
    yview = ybig[32:32 + n].reshape(shape)
    y = cz.decompress_host(s, shape, dtype, mb, out=yview)
    assert np.array_equal(y.view(np.uint32), want.view(np.uint32))
    assert np.all(ybig[:32] == 7.0) and np.all(ybig[32 + n:] == 7.0)


@pytest.mark.gpu
@pytest.mark.parametrize("dims", [1, 2, 3])
@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.int32, np.int64])
def test_random_streams(cuda, restatement, dims, dtype):
    """Arbitrary bit streams decoded on the GPU exactly as the reference decodes
    them: dense / sparse bit patterns reach every path of the plane decoder
    (chunked dense codes, the one implied at position N-1, the budget ending
    inside a run, the sequential fallback) in many lanes of a wave at once."""
    import torch
    rng = np.random.default_rng(31 + dims + 10 * np.dtype(dtype).itemsize)
    for trial in range(12):
        shape = tuple(int(rng.integers(1, 40 if dims < 3 else 20)) for _ in range(dims))
        if trial == 0:
            shape = (64,) * dims if dims < 3 else (32, 32, 32)
        mb = int(rng.choice([12, 33, 63, 64, 65, 127, 128, 191, 256, 512, 777, 1024, 2000]))
        nb = int(np.prod([(s + 3) // 4 for s in shape]))
        words = (nb * mb + 63) // 64
        density = (0.5, 0.1, 0.9, 0.03, 0.97, 0.7)[trial % 6]
        bits = rng.random(words * 64) < density
        s = np.packbits(bits.reshape(-1, 8)[:, ::-1], axis=1).reshape(-1).view(np.uint64).copy()
        want = restatement.decompress(s, shape, dtype, mb)
        d = torch.from_numpy(s.view(np.int64)).to(cuda)
        tdt = {np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64,
               np.dtype(np.int32): torch.int32, np.dtype(np.int64): torch.int64}[np.dtype(dtype)]
        got = cz.decode(d, shape, tdt, mb).cpu().numpy()
        assert np.array_equal(got.view(np.uint8), want.view(np.uint8)), (shape, mb, density)


# --------------------------------------------------------------------------
# persistent 1D/2D launches: more batches than resident waves (each wave codes
# several), a partial last batch, strided / padded fields on the same path


@pytest.mark.parametrize("dims,shape", [(1, (3 * 2 ** 20 + 7,)), (2, (2050, 1030)), (1, (5 * 2 ** 20,))])
@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.int32])
def test_persistent_batches(cuda, restatement, dims, shape, dtype):
    rng = np.random.default_rng(zlib.crc32(f"{dims}/{shape}/{np.dtype(dtype).str}".encode()))
    if np.dtype(dtype).kind == "i":
        a = rng.integers(-2 ** 24, 2 ** 24, size=shape).astype(dtype)
    else:
        a = _fields(rng, shape, dtype, "smooth")
    for rate in (3, 8, 21):
        mb = cz.rate_to_maxbits(rate, dtype, dims)
        words, y = _gpu_roundtrip(a, mb, cuda)
        ref = restatement.compress(a, mb)
        assert np.array_equal(words, ref), rate
        assert np.array_equal(y, restatement.decompress(ref, shape, dtype, mb)), rate


# --------------------------------------------------------------------------
# launches of several resident rounds of waves run the kernels without the
# plane-loop priority schedule (kernels.hpp, use_priority): encoder beyond one
# round, decoder beyond two (f32: 4,096 waves a round on 256 CUs; 3D f64: 2,048)


@pytest.mark.parametrize("shape,dtype,rate", [((576, 256, 256), np.float32, 8),
                                              ((288, 256, 256), np.float64, 16)])
def test_multi_round_3d(cuda, restatement, shape, dtype, rate):
    rng = np.random.default_rng(7)
    a = _fields(rng, shape, dtype, "smooth")
    mb = cz.rate_to_maxbits(rate, dtype, 3)
    words, y = _gpu_roundtrip(a, mb, cuda)
    ref = restatement.compress(a, mb)
    assert np.array_equal(words, ref)
    assert np.array_equal(y, restatement.decompress(ref, shape, dtype, mb))


# --------------------------------------------------------------------------
# blocks of at most 64 bits take the register reader (kernels.hpp, RegReader):
# every such maxbits class in 1D/2D, random streams of several densities and
# encoded fields, multi-wave arrays with a partial last wave


@pytest.mark.parametrize("dims", [1, 2])
@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.int32])
def test_register_reader(cuda, restatement, dims, dtype):
    import torch
    rng = np.random.default_rng(101 + dims + 7 * np.dtype(dtype).itemsize)
    tdt = {np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64,
           np.dtype(np.int32): torch.int32}[np.dtype(dtype)]
    shape = (4 * 64 * 5 + 9,) if dims == 1 else (90, 75)
    for mb in (9, 12, 13, 17, 31, 32, 33, 47, 48, 63, 64):
        if mb < (9 if np.dtype(dtype).itemsize == 4 else 12):
            continue
        nb = int(np.prod([(s + 3) // 4 for s in shape]))
        words = (nb * mb + 63) // 64
        for density in (0.5, 0.05, 0.95):
            bits = rng.random(words * 64) < density
            s = np.packbits(bits.reshape(-1, 8)[:, ::-1], axis=1).reshape(-1).view(np.uint64).copy()
            want = restatement.decompress(s, shape, dtype, mb)
            got = cz.decode(torch.from_numpy(s.view(np.int64)).to(cuda), shape, tdt, mb).cpu().numpy()
            assert np.array_equal(got.view(np.uint8), want.view(np.uint8)), (mb, density)
        if np.dtype(dtype).kind == "f":
            a = _fields(rng, shape, dtype, "smooth")
            w, y = _gpu_roundtrip(a, mb, cuda)
            ref = restatement.compress(a, mb)
            assert np.array_equal(w, ref), mb
            assert np.array_equal(y.view(np.uint8), restatement.decompress(ref, shape, dtype, mb).view(np.uint8)), mb


@pytest.mark.parametrize("mb", [32, 64])
@pytest.mark.parametrize("dims", [1, 2])
@pytest.mark.parametrize("dtype", [np.int32, np.int64])
def test_int_register_writer(cuda, restatement, dims, dtype, mb):
    """Integer blocks of 32 and 64 bits (1D / 2D): the register writer
    (RegWriter, FULL64 masking at 64) and register reader, against the
    restatement's block-level int32 / int64 coder; 1D at more than 32,768 waves
    as well (integer fields take the general-gather kernels at every size)."""
    rng = np.random.default_rng(mb + 10 * dims + np.dtype(dtype).itemsize)
    shapes = [(4 * 64 * 5 + 9,), (4 * 64 * 32769 + 6,)] if dims == 1 else [(90, 75), (1030, 517)]
    for shape in shapes:
        for kind in ("uniform", "smooth"):
            if kind == "uniform":
                a = rng.integers(-2 ** 24, 2 ** 24, size=shape).astype(dtype)
            else:
                a = np.cumsum(rng.integers(-1000, 1000, size=shape), axis=-1).astype(dtype)
            words, y = _gpu_roundtrip(a, mb, cuda)
            ref = restatement.compress(a, mb)
            assert np.array_equal(words, ref), (shape, kind)
            assert np.array_equal(y, restatement.decompress(ref, shape, dtype, mb)), (shape, kind)


@pytest.mark.parametrize("dims", [1, 2])
def test_register_writer_extremes(cuda, restatement, dims):
    """f32 blocks of 32 bits (1D rate 8, 2D rate 2: RegWriter32, which keeps
    stream bits 1..32 and relies on a coded block's first bit being one) and
    of 64 bits, on blocks that take every quantisation path: all-zero blocks
    (no exponent field), denormals and tiny exponents (the exact path, for the
    whole wave), huge values, inf and NaN, mixed with smooth blocks in the
    same waves; 1D also past 32,768 waves (the batched kernels)."""
    rng = np.random.default_rng(55 + dims)
    shapes = [(4 * 64 * 7 + 3,), (4 * 64 * 32769 + 2,)] if dims == 1 else [(90, 75), (260, 514)]
    for shape in shapes:
        a = _fields(rng, shape, np.float32, "smooth")
        flat = a.reshape(-1)
        n = flat.size
        idx = rng.permutation(n)
        k = n // 16
        flat[idx[:k]] = 0.0
        flat[idx[k:2 * k]] *= np.float32(1e-38)
        flat[idx[2 * k:3 * k]] = (rng.standard_normal(k) * 1e-44).astype(np.float32)
        with np.errstate(over="ignore"):
            flat[idx[3 * k:4 * k]] *= np.float32(3e37)
        flat[idx[4 * k:4 * k + 50]] = np.inf
        flat[idx[4 * k + 50:4 * k + 100]] = -np.inf
        flat[idx[4 * k + 100:4 * k + 150]] = np.nan
        if dims == 1:
            flat[: 4 * 64] = 0.0  # a whole wave of zero blocks
        else:
            a[:8, :] = 0.0
        for mb in (32, 64):
            words, y = _gpu_roundtrip(a, mb, cuda)
            ref = restatement.compress(a, mb)
            assert np.array_equal(words, ref), (shape, mb)
            assert np.array_equal(y.view(np.uint8), restatement.decompress(ref, shape, np.float32, mb).view(np.uint8)), (shape, mb)


def test_f64_staged_rows(cuda, restatement):
    """3D double decodes whose waves are whole x-row segments (256 wide: 64
    blocks) store their rows through the wave's LDS image (kernels.hpp,
    scatter_f64_staged: 4, 2 or 1 rows a pass by maxbits, none below), with
    zero blocks among coded ones in the same waves."""
    rng = np.random.default_rng(64)
    a = _fields(rng, (8, 12, 256), np.float64, "smooth")
    a[:, :4, :64] = 0.0      # zero blocks in a wave's first half
    a[4:, 4:8, 192:] = 0.0   # ... and in its last quarter
    for rate in (16, 8, 2, 1, 40):
        mb = cz.rate_to_maxbits(rate, np.float64, 3)
        words, y = _gpu_roundtrip(a, mb, cuda)
        ref = restatement.compress(a, mb)
        assert np.array_equal(words, ref), rate
        assert np.array_equal(y.view(np.uint8), restatement.decompress(ref, a.shape, np.float64, mb).view(np.uint8)), rate


@pytest.mark.parametrize("dtype,mb", [(np.float32, 384), (np.float32, 640), (np.float64, 768), (np.float64, 1152)])
def test_lane_order_non_pow2_words(cuda, restatement, dtype, mb):
    """The full-wave lane-order stream copies (kernels.hpp: the encoder's
    copy-out over W = maxbits/64 words a block, the decoder's copy-in over D =
    maxbits/32 dwords) with W and D even but not powers of two, which takes
    udivmod_uniform's division branch: 16 full 64-block waves of
    a fixed-seed field, smooth and rough halves, against the restatement."""
    rng = np.random.default_rng(384 + mb)
    a = _fields(rng, (16, 16, 256), dtype, "smooth")
    a[8:] = _fields(rng, (8, 16, 256), dtype, "normal")
    words, y = _gpu_roundtrip(a, mb, cuda)
    ref = restatement.compress(a, mb)
    assert np.array_equal(words, ref), mb
    assert np.array_equal(y.view(np.uint8), restatement.decompress(ref, a.shape, dtype, mb).view(np.uint8)), mb


@pytest.mark.parametrize("nblocks", [64 * 32771, 64 * 32769 + 25, 64 * 32768 - 1])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_batched_1d_waves(cuda, restatement, nblocks, dtype):
    """1D launches of >= 32,768 waves take the batched register-path kernels
    (kernels.hpp zfp_encode_regk / zfp_decode_regk: 2 and 4 batches of 64 blocks
    a wave): a last wave group with fewer batches, a partial last batch, and the
    size just below the switch (the one-batch kernels)."""
    rng = np.random.default_rng(nblocks % 1000)
    shape = (4 * nblocks,)
    a = _fields(rng, shape, dtype, "smooth")
    for rate in (3, 8, 16):
        mb = cz.rate_to_maxbits(rate, dtype, 1)
        words, y = _gpu_roundtrip(a, mb, cuda)
        ref = restatement.compress(a, mb)
        assert np.array_equal(words, ref), rate
        assert np.array_equal(y.view(np.uint8), restatement.decompress(ref, shape, dtype, mb).view(np.uint8)), rate


@pytest.mark.parametrize("shape,dtype,rate", [((64, 48, 40), np.float32, 8), ((24, 20, 16), np.float64, 16),
                                              ((300, 260), np.float32, 4), ((200003,), np.float32, 8)])
@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("ordered,zero_copy", [("0", "0"), ("1", "0"), ("1", "2")])
def test_host_pipeline_multi_chunk(cuda, restatement, monkeypatch, shape, dtype, rate, pinned, ordered, zero_copy):
    """The host pipeline with chunks far smaller than the array
    (CUZFP_HOST_CHUNK_BYTES): waves straddling chunks, the cross-stream event
    waits and the pageable staging ring, for 1, 2 and 3 streams, in both
    schedules (CUZFP_HOST_ORDERED), with the kernels addressing pinned buffers
    themselves (CUZFP_HOST_ZEROCOPY=2: compression in one launch, decode
    kernels storing to the array) or not (0)."""
    import torch
    monkeypatch.setenv("CUZFP_HOST_ORDERED", ordered)
    monkeypatch.setenv("CUZFP_HOST_ZEROCOPY", zero_copy)
    from cuzfp_amd.datagen import splitmix_uniform
    a = splitmix_uniform(shape, dtype, seed=9)
    mb = cz.rate_to_maxbits(rate, dtype, len(shape))
    ref = restatement.compress(a, mb)
    want = restatement.decompress(ref, shape, dtype, mb)
    out = None
    if pinned:
        a = torch.from_numpy(a).pin_memory().numpy()
        out = torch.empty(cz.stream_bytes(shape, dtype, mb) // 8, dtype=torch.int64).pin_memory().numpy().view(np.uint64)
    yout = torch.empty(shape, dtype=torch.from_numpy(a).dtype).pin_memory().numpy() if pinned else None
    slab = a.nbytes // (shape[0] // 4 if len(shape) > 1 else max(1, shape[0] // 4))
    # 8 slabs a chunk and a.nbytes // 7 (1D, 2D) run the ordered schedule's
    # growing edge chunks (capi.hip host_pipeline); pinned buffers both ways
    # its three-pass queue filling
    for chunk in (1, 3 * slab + 5, 8 * slab, a.nbytes // 7):
        monkeypatch.setenv("CUZFP_HOST_CHUNK_BYTES", str(chunk))
        for nstreams in (1, 2, 3):
            s = cz.compress_host(a, mb, nstreams=nstreams, out=out)
            assert np.array_equal(s, ref), (chunk, nstreams)
            y = cz.decompress_host(s, shape, dtype, mb, nstreams=nstreams)
            assert np.array_equal(y, want), (chunk, nstreams)
            if pinned:
                yout.fill(7)
                y = cz.decompress_host(s, shape, dtype, mb, nstreams=nstreams, out=yout)
                assert np.array_equal(y, want), (chunk, nstreams, "pinned out")


def test_broadcast_view_encodes_materialised(cuda, restatement):
    """An expanded tensor (a zero stride) encodes as its materialised copy;
    decoding into a broadcast view is refused."""
    import torch
    base = torch.linspace(-1, 1, 16, dtype=torch.float32, device=cuda)
    x = base.expand(12, 16)
    mb = cz.rate_to_maxbits(8, np.float32, 2)
    w = cz.encode(x, mb)
    ref = restatement.compress(np.ascontiguousarray(x.cpu().numpy()), mb)
    assert np.array_equal(w.cpu().numpy().view(np.uint64), ref)
    with pytest.raises(ValueError):
        cz.decode(w, (12, 16), torch.float32, mb, out=torch.empty(16, dtype=torch.float32, device=cuda).expand(12, 16))


def test_host_cache_release(cuda, restatement):
    """The host pipeline's retained buffers are freed by release_host_cache and
    rebuilt by the next call; results are unchanged, pageable staging included."""
    from cuzfp_amd.datagen import splitmix_uniform
    a = splitmix_uniform((40, 36, 28), np.float32, seed=9)
    mb = cz.rate_to_maxbits(8, np.float32, 3)
    ref = restatement.compress(a, mb)
    for _ in range(2):
        s = cz.compress_host(a, mb)
        assert np.array_equal(s, ref)
        assert np.array_equal(cz.decompress_host(s, a.shape, np.float32, mb),
                              restatement.decompress(ref, a.shape, np.float32, mb))
        cz.release_host_cache()
    cz.release_host_cache(0)  # twice in a row: a no-op


def test_broadcast_view_side_stream(cuda, restatement):
    """A broadcast view encoded on a side stream: the materialising copy runs on
    that stream after the current stream's pending work (here the kernel that
    writes the base tensor), and the base stays allocated until that copy has
    read it (record_stream on the side stream).  The side stream is held back by
    a spin kernel, so without the record a same-size allocation on the current
    stream reuses the freed base and overwrites it with NaNs before the copy."""
    import torch
    side = torch.cuda.Stream(device=cuda)
    mb = cz.rate_to_maxbits(8, np.float32, 3)
    for trial in range(4):
        base = torch.empty(64, dtype=torch.float32, device=cuda)
        # exact values (power-of-two scale), written by a kernel queued on the current stream
        base.copy_(torch.arange(64, dtype=torch.float32, device=cuda) * (trial + 1) / 64 - 0.5)
        with torch.cuda.stream(side):
            torch.cuda._sleep(20_000_000)  # the side stream's copy runs well after the lines below
        x = base.expand(40, 32, 64)
        w = cz.encode(x, mb, stream=side)
        del x, base
        junk = torch.empty(64, dtype=torch.float32, device=cuda)  # base's size class, current stream
        junk.fill_(float("nan"))
        side.synchronize()
        torch.cuda.synchronize()
        vals = np.arange(64, dtype=np.float32) * np.float32(trial + 1) / np.float32(64) - np.float32(0.5)
        ref = restatement.compress(np.broadcast_to(vals, (40, 32, 64)).copy(), mb)
        assert np.array_equal(w.cpu().numpy().view(np.uint64), ref), trial
        del junk


def test_copy_checks(cuda):
    """cz.copy() refuses non-contiguous and host tensors."""
    import torch
    a = torch.zeros(64, 2, dtype=torch.float32, device=cuda)
    with pytest.raises(ValueError):
        cz.copy(a.t(), torch.empty(128, device=cuda))
    with pytest.raises(ValueError):
        cz.copy(torch.zeros(16), torch.empty(16, device=cuda))
    b = torch.arange(1 << 12, dtype=torch.float32, device=cuda)
    c = torch.empty_like(b)
    cz.copy(b, c)
    torch.cuda.synchronize()
    assert torch.equal(b, c)


@pytest.mark.parametrize("dims,dtype", [(3, np.float64), (3, np.float32), (2, np.float64), (1, np.float32)])
def test_largest_maxbits(cuda, restatement, dims, dtype):
    """maxbits at the cap (CUZFP_MAX_BITS = 16384, sized for gfx950's 160 KiB of
    LDS a workgroup): the widest LDS stream images (one wave per workgroup,
    dynamic LDS past 64 KiB) against the oracle, and the old 64 KiB cap."""
    from cuzfp_amd.datagen import splitmix_uniform
    shape = {1: (1000,), 2: (36, 28), 3: (12, 8, 20)}[dims]
    a = splitmix_uniform(shape, dtype, seed=3)
    for mb in (16384, 16383, 9999, 6144, 4171):
        words, y = _gpu_roundtrip(a, mb, cuda)
        ref = restatement.compress(a, mb)
        assert np.array_equal(words, ref), mb
        assert np.array_equal(y, restatement.decompress(ref, shape, dtype, mb)), mb


def _golden_1024():
    import json
    import os
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden.json")
    return json.load(open(path))["cases"]["baseline/3d_f32_1024_r8/polynomial"]


@pytest.mark.timeout(600)
def test_golden_1024_full_array(cuda):
    """BASELINE configs[4]'s whole 1024^3 array on one GPU: the stream and the
    decoded array against the reference's SHA-256s (tests/golden/golden.json,
    made from the compiled reference by make_golden.py)."""
    import hashlib
    import torch
    from cuzfp_amd.datagen import polynomial_slab_device
    gold = _golden_1024()
    x = polynomial_slab_device((1024, 1024, 1024), 0, 1024, cuda)
    mb = cz.rate_to_maxbits(8, np.float32, 3)
    words = cz.encode(x, mb)
    y = cz.decode(words, x.shape, x.dtype, mb)
    torch.cuda.synchronize()
    assert hashlib.sha256(words.cpu().numpy().tobytes()).hexdigest() == gold["stream_sha256"]
    del x, words
    assert hashlib.sha256(y.cpu().numpy().tobytes()).hexdigest() == gold["decoded_sha256"]


@pytest.mark.parametrize("world,rank", [(8, 0), (8, 7), (4, 2), (2, 1)])
def test_golden_1024_slab(cuda, world, rank):
    """One rank's z-slab of the 1024^3 array (1024/N planes) encodes to exactly
    its word range of the reference's stream: [r*W/N, (r+1)*W/N)."""
    import hashlib
    import torch
    from cuzfp_amd import dist as zd
    from cuzfp_amd.datagen import polynomial_slab_device
    gold = _golden_1024()
    mb = cz.rate_to_maxbits(8, np.float32, 3)
    sh = zd.StrongShard(1024, world, rank, mb)
    x = polynomial_slab_device(sh.global_shape, sh.z0, sh.z1, cuda)
    words = cz.encode(x, mb)
    torch.cuda.synchronize()
    assert words.numel() == sh.words
    assert hashlib.sha256(words.cpu().numpy().tobytes()).hexdigest() == gold[f"slab_sha256_n{world}"][rank]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [np.float64, np.int64])
def test_split_transpose_64bit(cuda, restatement, dtype):
    """The 3D 64-bit encoder's low-half planes, transposed 16 at a time only
    while some lane of the wave has budget (zfp_block.hpp, planes::load_split):
    rates that stop waves above plane 32, between 32 and 16 and below 16, in
    aligned (lane-interleaved image) arrays, with waves mixing blocks of every
    magnitude and, for doubles, tiny-exponent blocks (maxprec < 64: the rolled
    path after the split transpose) beside normal ones."""
    rng = np.random.default_rng(641)
    shape = (8, 16, 256)  # whole waves of 64 blocks along x
    if dtype == np.float64:
        a = np.cumsum(rng.standard_normal(shape), axis=-1) * 10.0 ** rng.integers(-8, 8, size=shape)
        a[:4, :4, :128] *= 1e-310  # tiny-exponent blocks in some waves
    else:
        a = (np.cumsum(rng.integers(-1 << 40, 1 << 40, size=shape), axis=-1) >> rng.integers(0, 40, size=shape))
    a = a.astype(dtype)
    for rate in (2, 6, 12, 20, 28, 36, 48, 64):
        mb = cz.rate_to_maxbits(rate, dtype, 3)
        words, y = _gpu_roundtrip(a, mb, cuda)
        ref = restatement.compress(a, mb)
        assert np.array_equal(words, ref), rate
        assert np.array_equal(y.view(np.uint8), restatement.decompress(ref, a.shape, dtype, mb).view(np.uint8)), rate
