"""Host emulation of the GPU lane algorithm (CPU-only).

tests/native/emulate.cpp runs cuzfp_amd/csrc/zfp_block.hpp -- the exact
per-lane functions every GPU lane executes -- on the host.  Checking it
against the oracle here validates the block coder (exponent, quantisation,
lifting, permutation, bit-plane transpose, embedded coder, window reader)
without a GPU; tests/test_gpu_parity.py then checks the kernels themselves.
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "emulate.cpp")
HDR = os.path.join(ROOT, "cuzfp_amd", "csrc", "zfp_block.hpp")
HOST_IO = os.path.join(ROOT, "tests", "native", "host_io.hpp")
LIB = os.path.join(ROOT, "build", "libcuzfp_emu.so")
TC = {np.dtype(np.int32): 1, np.dtype(np.int64): 2, np.dtype(np.float32): 3, np.dtype(np.float64): 4}


@pytest.fixture(scope="module")
def emu():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(f) for f in (SRC, HDR, HOST_IO)):
        subprocess.check_call(["/opt/rocm/llvm/bin/clang++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wno-unknown-pragmas",
                               "-o", LIB, SRC])
    lib = ctypes.CDLL(LIB)
    args = [ctypes.c_int] + [ctypes.c_uint] * 3 + [ctypes.c_longlong] * 3 + [ctypes.c_uint]
    lib.emu_compress.restype = ctypes.c_size_t
    lib.emu_compress.argtypes = args + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    lib.emu_decompress.restype = ctypes.c_int
    lib.emu_decompress.argtypes = args + [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    return lib


def _ext(shape):
    padded = tuple(shape[::-1]) + (0, 0)
    return padded[0], padded[1], padded[2]


def emu_compress(lib, a, mb):
    nx, ny, nz = _ext(a.shape)
    nb = int(np.prod([(s + 3) // 4 for s in a.shape]))
    cap = ((nb * mb + 63) // 64) * 8
    out = np.zeros(max(cap, 8) // 8, np.uint64)
    n = lib.emu_compress(TC[a.dtype], nx, ny, nz, 0, 0, 0, mb, a.ctypes.data, out.ctypes.data, out.nbytes)
    assert n == cap
    return out[: n // 8]


def emu_decompress(lib, s, shape, dtype, mb):
    nx, ny, nz = _ext(shape)
    out = np.zeros(shape, dtype)
    assert lib.emu_decompress(TC[np.dtype(dtype)], nx, ny, nz, 0, 0, 0, mb, s.ctypes.data, s.nbytes,
                              out.ctypes.data)
    return out


def _rand(rng, shape, dtype, kind):
    if kind == 0:
        a = rng.standard_normal(shape)
    elif kind == 1:
        a = np.cumsum(rng.standard_normal(shape), axis=-1)
    elif kind == 2:
        a = rng.standard_normal(shape) * 10.0 ** rng.integers(-40, 40, size=shape)
    else:
        a = np.where(rng.random(shape) < 0.5, 0, rng.standard_normal(shape))
    with np.errstate(over="ignore"):
        return a.astype(dtype)


@pytest.mark.parametrize("dims", [1, 2, 3])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_emulation_vs_oracle(emu, restatement, dims, dtype):
    rng = np.random.default_rng(100 + dims * 2 + (dtype == np.float64))
    for trial in range(30):
        shape = tuple(int(rng.integers(1, 40 if dims < 3 else 14)) for _ in range(dims))
        a = _rand(rng, shape, dtype, trial % 4)
        rate = float(rng.integers(1, 33)) if trial % 3 else float(rng.uniform(0.5, 64))
        mb = restatement.rate_to_maxbits(rate, dtype, dims)
        s = restatement.compress(a, mb)
        assert np.array_equal(emu_compress(emu, a, mb), s), (shape, mb)
        d = emu_decompress(emu, s, shape, dtype, mb)
        assert np.array_equal(d.view(np.uint8), restatement.decompress(s, shape, dtype, mb).view(np.uint8))


@pytest.mark.parametrize("dims", [1, 2, 3])
@pytest.mark.parametrize("dtype", [np.int32, np.int64])
def test_emulation_int(emu, restatement, dims, dtype):
    rng = np.random.default_rng(dims)
    for trial in range(8):
        shape = tuple(int(rng.integers(1, 30 if dims < 3 else 10)) for _ in range(dims))
        lim = 2 ** (20 if trial % 2 else 30)
        a = rng.integers(-lim, lim, size=shape).astype(dtype)
        mb = int(rng.integers(2, 3000))
        s = restatement.compress(a, mb)
        assert np.array_equal(emu_compress(emu, a, mb), s)
        assert np.array_equal(emu_decompress(emu, s, shape, dtype, mb), restatement.decompress(s, shape, dtype, mb))


def test_emulation_extremes(emu, restatement):
    """denormal-only blocks, tiny blocks (x86 INT_MIN cast), inf, zeros, max maxbits."""
    rng = np.random.default_rng(5)
    cases = []
    for dt, scales in ((np.float32, [1e-30, 1e-38, 1e-44, 3e38]), (np.float64, [1e-300, 1e-310, 1e-320, 1e308])):
        for sc in scales:
            a = (rng.standard_normal((8, 8, 8)) * sc).astype(dt)
            a.flat[::5] = 0
            cases.append(a)
        z = np.zeros((8, 8, 8), dt)
        cases.append(z)
        inf = rng.standard_normal((8, 8, 8)).astype(dt)
        inf[0, 0, 0] = np.inf
        cases.append(inf)
    for a in cases:
        for mb in (restatement.rate_to_maxbits(1, a.dtype, 3), 512, 1000, 4171):
            s = restatement.compress(a, mb)
            assert np.array_equal(emu_compress(emu, a, mb), s)
            d = emu_decompress(emu, s, a.shape, a.dtype, mb)
            assert np.array_equal(d.view(np.uint8), restatement.decompress(s, a.shape, a.dtype, mb).view(np.uint8))


@pytest.mark.parametrize("dims", [1, 2, 3])
@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.int32, np.int64])
def test_emulation_random_streams(emu, restatement, dims, dtype):
    """Arbitrary bit streams (not encoder output) decoded the reference's way:
    dense and sparse bit patterns drive the decoder through every path of its
    plane step -- chunked dense codes, the one implied at position N-1, the
    budget ending inside a run (decode.c:311), the sequential fallback."""
    rng = np.random.default_rng(7 + dims + 10 * np.dtype(dtype).itemsize)
    for trial in range(24):
        shape = tuple(int(rng.integers(1, 24 if dims < 3 else 12)) for _ in range(dims))
        mb = int(rng.choice([12, 33, 63, 64, 65, 127, 128, 191, 256, 512, 777, 1024, 2000]))
        if np.dtype(dtype) == np.float64 and mb < 12:
            mb = 12
        nb = int(np.prod([(s + 3) // 4 for s in shape]))
        words = (nb * mb + 63) // 64
        density = (0.5, 0.1, 0.9, 0.03, 0.97, 0.7)[trial % 6]
        bits = rng.random(words * 64) < density
        s = np.packbits(bits.reshape(-1, 8)[:, ::-1], axis=1).reshape(-1).view(np.uint64).copy()
        want = restatement.decompress(s, shape, dtype, mb)
        got = emu_decompress(emu, s, shape, dtype, mb)
        assert np.array_equal(got.view(np.uint8), want.view(np.uint8)), (shape, mb, density)


@pytest.mark.parametrize("dims", [1, 2, 3])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_emulation_large_maxbits(emu, restatement, dims, dtype):
    """Budgets past 2^13 (up to CUZFP_MAX_BITS = 16384, which the LDS of a
    gfx950 workgroup allows): dense random streams make the plane decoder's
    running bit counts pass the chunk entries' "not ended" marker (2^13), and
    fields at those maxbits run every plane with budget to spare."""
    from cuzfp_amd.datagen import splitmix_uniform
    rng = np.random.default_rng(31 + dims)
    shape = {1: (40,), 2: (12, 8), 3: (8, 4, 8)}[dims]
    nb = int(np.prod([(s + 3) // 4 for s in shape]))
    for mb in (8191, 8193, 9999, 16383, 16384):
        for density in (0.5, 0.9, 0.97):
            words = (nb * mb + 63) // 64
            bits = rng.random(words * 64) < density
            s = np.packbits(bits.reshape(-1, 8)[:, ::-1], axis=1).reshape(-1).view(np.uint64).copy()
            want = restatement.decompress(s, shape, dtype, mb)
            got = emu_decompress(emu, s, shape, dtype, mb)
            assert np.array_equal(got.view(np.uint8), want.view(np.uint8)), (mb, density)
        a = splitmix_uniform(shape, dtype, seed=mb)
        s = restatement.compress(a, mb)
        assert np.array_equal(emu_compress(emu, a, mb), s), mb
        got = emu_decompress(emu, s, shape, dtype, mb)
        assert np.array_equal(got.view(np.uint8), restatement.decompress(s, shape, dtype, mb).view(np.uint8)), mb


@pytest.mark.parametrize("dims", [1, 2, 3])
def test_emulation_budget_cuts(emu, restatement, dims):
    """Encoder output at every rate 1..32 (so the budget ends at every offset
    of the table decoder's window), smooth, noisy and rough fields: the table
    decoder's budget-cut and position-63 cases against the oracle."""
    from cuzfp_amd.datagen import polynomial_field, splitmix_uniform
    shape = {1: (4096,), 2: (64, 64), 3: (16, 16, 32)}[dims]
    rng = np.random.default_rng(11 + dims)
    fields = [polynomial_field(shape, np.float32), splitmix_uniform(shape, np.float32),
              (polynomial_field(shape, np.float32) + 1e-3 * rng.standard_normal(shape)).astype(np.float32)]
    for a in fields:
        for rate in range(1, 33):
            mb = restatement.rate_to_maxbits(rate, a.dtype, dims)
            s = restatement.compress(a, mb)
            assert np.array_equal(emu_compress(emu, a, mb), s), rate
            got = emu_decompress(emu, s, a.shape, a.dtype, mb)
            assert np.array_equal(got.view(np.uint8), restatement.decompress(s, a.shape, a.dtype, mb).view(np.uint8)), rate


@pytest.mark.parametrize("dims", [1, 2, 3])
def test_table_plane_decoder_fuzz(emu, dims):
    """One plane step from random decoder states (n, budget, stream bits of
    every density, the stream zero past the budget): the table decoder the
    kernels run must equal the general decoder bit for bit."""
    emu.emu_fuzz_plane.restype = ctypes.c_longlong
    emu.emu_fuzz_plane.argtypes = [ctypes.c_ulonglong, ctypes.c_longlong, ctypes.c_int]
    assert emu.emu_fuzz_plane(1234 + dims, 2_000_000, dims) == 0


def test_block_index_division_magic(tmp_path):
    """The launch's multiply-shift division of block indices (launch.hpp
    set_divisor, used by block_pos for n < 2^31) equals integer division."""
    exe = str(tmp_path / "divmagic")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-o", exe,
                           os.path.join(ROOT, "tests", "native", "divmagic.cpp")])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "0", out.stdout + out.stderr

