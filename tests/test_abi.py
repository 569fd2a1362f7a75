"""The C-ABI boundary (CPU-only: no kernel launches).

* libcuzfp_hip.so loads and exports every function include/cuzfp_hip.h declares;
* libcuZFP.so exports the reference's C++ entry points cuZFP::compress /
  cuZFP::decompress (src/cuZFP/cuZFP.h:9-10);
* the host-only helpers agree with the oracle / reference formulas;
* argument errors come back as status codes before any device work.
"""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import cuzfp_amd as cz

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "cuzfp_hip.h")


@pytest.fixture(scope="module")
def libs():
    from cuzfp_amd.build import build
    return build()


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(cuzfp_hip_\w+)\s*\(", text)))


def exported(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_header_symbols_exported(libs):
    syms = exported(libs["hip"])
    names = declared_functions()
    assert len(names) >= 10
    missing = [n for n in names if n not in syms]
    assert not missing, missing


def test_release_host_cache_bad_device(libs):
    """cuzfp_hip_release_host_cache rejects device ordinals outside its cache
    before touching the runtime (no GPU needed)."""
    lib = cz.library()
    assert lib.cuzfp_hip_release_host_cache(99) == 1
    assert lib.cuzfp_hip_release_host_cache(-2) == 1


def test_cpp_dropin_symbols(libs):
    out = subprocess.run(["nm", "-DC", "--defined-only", libs["cpp"]], capture_output=True, text=True).stdout
    assert "cuZFP::compress(cuZFP::zfp_stream*, cuZFP::zfp_field*)" in out
    assert "cuZFP::decompress(cuZFP::zfp_stream*, cuZFP::zfp_field*)" in out


def test_library_loads(libs):
    lib = cz.library()
    assert lib.cuzfp_hip_abi_version() == 1
    assert lib.cuzfp_hip_status_string(0) == b"success"
    assert lib.cuzfp_hip_status_string(3) == b"stream buffer too small"


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_rate_to_maxbits_matches_zfp(libs, restatement, dtype):
    for dims in (1, 2, 3):
        for rate in (0.25, 1, 1.5, 2, 7.9, 8, 16, 31, 64):
            for wra in (False, True):
                assert cz.rate_to_maxbits(rate, dtype, dims, wra) == restatement.rate_to_maxbits(rate, dtype, dims, wra)


def test_stream_bytes(libs, restatement):
    for shape in [(1,), (5,), (1 << 20,), (3, 7), (8192, 8192), (1, 1, 1), (13, 17, 19), (256, 256, 256)]:
        for mb in (9, 32, 100, 512, 1024):
            assert cz.stream_bytes(shape, np.float32, mb) == restatement.stream_bytes(shape, mb)


def test_maximum_size(libs, reference):
    for shape in [(100,), (64, 64), (16, 8, 4), (13, 17, 19)]:
        for dt, mb in ((np.float32, 512), (np.float64, 1024), (np.float32, 4171)):
            nx, ny, nz = (tuple(shape[::-1]) + (0, 0))[:3]
            want = reference.lib.ref_maximum_size
            want.restype = ctypes.c_size_t
            want.argtypes = [ctypes.c_int] + [ctypes.c_uint] * 4
            got = cz.maximum_size(shape, dt, mb)
            assert got >= cz.stream_bytes(shape, dt, mb)
            # zfp_stream_maximum_size with minbits == maxbits (fixed rate)
            assert got == want(3 if dt == np.float32 else 4, nx, ny, nz, mb)


def test_argument_errors(libs):
    lib = cz.library()
    got = ctypes.c_size_t(0)
    buf = ctypes.c_void_p(0x1000)  # never dereferenced: rejected before any launch
    # unsupported type
    assert lib.cuzfp_hip_encode(buf, 9, 16, 16, 16, 0, 0, 0, 512, buf, 1 << 20, ctypes.byref(got), None) == 2
    # nz without ny, nx == 0
    assert lib.cuzfp_hip_encode(buf, 3, 16, 0, 16, 0, 0, 0, 512, buf, 1 << 20, ctypes.byref(got), None) == 1
    assert lib.cuzfp_hip_encode(buf, 3, 0, 0, 0, 0, 0, 0, 512, buf, 1 << 20, ctypes.byref(got), None) == 1
    # maxbits below the exponent header
    assert lib.cuzfp_hip_encode(buf, 3, 16, 16, 16, 0, 0, 0, 8, buf, 1 << 20, ctypes.byref(got), None) == 1
    assert lib.cuzfp_hip_encode(buf, 4, 16, 16, 16, 0, 0, 0, 11, buf, 1 << 20, ctypes.byref(got), None) == 1
    # stream too small
    assert lib.cuzfp_hip_encode(buf, 3, 16, 16, 16, 0, 0, 0, 512, buf, 100, ctypes.byref(got), None) == 3
    assert lib.cuzfp_hip_decode(buf, 100, 3, 16, 16, 16, 0, 0, 0, 512, buf, None) == 3
    # null pointers
    assert lib.cuzfp_hip_encode(None, 3, 16, 16, 16, 0, 0, 0, 512, buf, 1 << 20, ctypes.byref(got), None) == 1
    assert lib.cuzfp_hip_compress_host(None, 3, 16, 16, 16, 512, buf, 1 << 20, ctypes.byref(got), 2) == 1
    with pytest.raises(cz.CodecError):
        cz.stream_bytes((16, 16, 16), np.float32, 3)


def test_maxbits_cap(libs):
    """maxbits up to CUZFP_MAX_BITS (16384, far above zfp's ZFP_MAX_BITS = 4171)
    is accepted; above it every entry point rejects the call (the decoder's LDS
    stream image would no longer fit a gfx950 workgroup's 160 KiB)."""
    lib = cz.library()
    cap = int(re.search(r"#define CUZFP_MAX_BITS (\d+)", open(HEADER).read()).group(1))
    assert cap == 16384
    assert cz.stream_bytes((16, 16, 16), np.float64, cap) == 64 * cap // 8
    with pytest.raises(cz.CodecError):
        cz.stream_bytes((16, 16, 16), np.float64, cap + 1)
    got = ctypes.c_size_t(0)
    buf = ctypes.c_void_p(0x1000)  # never dereferenced: rejected before any launch
    assert lib.cuzfp_hip_encode(buf, 4, 16, 16, 16, 0, 0, 0, cap + 1, buf, 1 << 30, ctypes.byref(got), None) == 1
    assert lib.cuzfp_hip_decode(buf, 1 << 30, 4, 16, 16, 16, 0, 0, 0, cap + 1, buf, None) == 1
    assert lib.cuzfp_hip_maximum_size(3, 16, 16, 16, cap + 1) == 0


def test_lds_budget_refusal(libs):
    """On a device with less LDS a workgroup (CUZFP_LDS_CAP_BYTES forces 64 KiB,
    read once a process) a block image that cannot fit beside the tables is
    refused with CUZFP_ERROR_INVALID_ARGUMENT before any launch (the
    launchers used to go ahead with one wave a workgroup and fail as a HIP
    error).  Fake pointers: the refusal comes before anything touches them."""
    code = r"""
import ctypes, sys
sys.path.insert(0, %r)
import cuzfp_amd as cz
lib = cz.library()
got = ctypes.c_size_t(0)
buf = ctypes.c_void_p(0x1000)
out = []
for t, dims in ((3, (16, 16, 16)), (4, (16, 16, 16)), (3, (64, 64, 0)), (3, (256, 0, 0))):
    nx, ny, nz = dims
    out.append(lib.cuzfp_hip_encode(buf, t, nx, ny, nz, 0, 0, 0, 16384, buf, 1 << 30, ctypes.byref(got), None))
    out.append(lib.cuzfp_hip_decode(buf, 1 << 30, t, nx, ny, nz, 0, 0, 0, 16384, buf, None))
print(out)
""" % ROOT
    env = dict(os.environ, CUZFP_LDS_CAP_BYTES="65536")
    r = subprocess.run([os.sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == str([1] * 8), r.stdout


def test_host_out_checks(libs):
    """compress_host / decompress_host validate a caller's `out` before the
    C side writes through it (contiguity, dtype, shape, size)."""
    a = np.zeros((8, 8, 8), np.float32)
    mb = 512
    need = cz.stream_bytes(a.shape, a.dtype, mb)
    with pytest.raises(ValueError):
        cz.compress_host(a, mb, out=np.empty(need // 8 - 1, np.uint64))
    with pytest.raises(ValueError):
        cz.compress_host(a, mb, out=np.empty(2 * (need // 8), np.uint64)[::2])
    words = np.zeros(need // 8, np.uint64)
    with pytest.raises(ValueError):
        cz.decompress_host(words, a.shape, np.float32, mb, out=np.empty((8, 8, 8), np.float64))
    with pytest.raises(ValueError):
        cz.decompress_host(words, a.shape, np.float32, mb, out=np.empty((8, 8, 16), np.float32)[:, :, ::2])
    with pytest.raises(ValueError):
        cz.decompress_host(words, a.shape, np.float32, mb, out=np.empty((8, 8, 4), np.float32))


def test_broadcast_views_detected():
    torch = pytest.importorskip("torch")
    assert cz._broadcast(torch.zeros(4).expand(8, 4))
    assert cz._broadcast(torch.zeros(1, 4).expand(3, 4))
    assert not cz._broadcast(torch.zeros(8, 4))
    assert not cz._broadcast(torch.zeros(1, 4))  # stride is irrelevant on an axis of extent 1
    assert not cz._broadcast(torch.zeros(8, 8)[:, ::2])
