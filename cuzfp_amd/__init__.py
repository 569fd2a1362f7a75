"""cuzfp_amd -- MI355X-native zfp fixed-rate codec (drop-in for mclarsen/cuZFP).

The codec is hand-written HIP for gfx950 (``cuzfp_amd/csrc``), exposed through
the C-ABI of ``include/cuzfp_hip.h`` (``lib/libcuzfp_hip.so``) and the
reference's C++ surface ``cuZFP::compress / decompress`` (``lib/libcuZFP.so``).
This module is the Python binding of that C-ABI; PyTorch provides device
memory and streams only.  There is no CPU fallback: every entry point raises
if the HIP library is missing.

Array shapes are numpy/torch order (slowest first): ``(nx,)``, ``(ny, nx)``,
``(nz, ny, nx)`` -- the reference's ``a[nz][ny][nx]`` (zfp_structs.h:42).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

__all__ = [
    "TYPE_INT32", "TYPE_INT64", "TYPE_FLOAT", "TYPE_DOUBLE", "CodecError",
    "library", "library_path", "rate_to_maxbits", "stream_bytes", "maximum_size",
    "encode", "decode", "compress_host", "decompress_host", "type_code",
]

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(HERE, "lib")

TYPE_INT32, TYPE_INT64, TYPE_FLOAT, TYPE_DOUBLE = 1, 2, 3, 4
_NP_TYPES = {np.dtype(np.int32): 1, np.dtype(np.int64): 2,
             np.dtype(np.float32): 3, np.dtype(np.float64): 4}
_STATUS = {0: "success", 1: "invalid argument", 2: "unsupported scalar type",
           3: "stream buffer too small", 4: "HIP runtime error"}


class CodecError(RuntimeError):
    """A non-zero cuzfp_status from the C-ABI."""

    def __init__(self, where: str, status: int, hip_error: int = 0):
        msg = f"{where}: {_STATUS.get(status, status)}"
        if status == 4:
            msg += f" (hipError {hip_error})"
        super().__init__(msg)
        self.status = status


_lib = None


def library_path() -> str:
    """The in-tree build; CUZFP_HIP_LIB overrides it (A/B runs of kernel variants)."""
    return os.environ.get("CUZFP_HIP_LIB") or os.path.join(LIB_DIR, "libcuzfp_hip.so")


def library() -> ctypes.CDLL:
    """Load ``libcuzfp_hip.so`` (built by ``cuzfp_amd/build.py``); raise if absent."""
    global _lib
    if _lib is not None:
        return _lib
    path = library_path()
    if not os.path.exists(path):
        raise RuntimeError(f"cuzfp_amd: HIP codec library not built ({path}); "
                           "run `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(path)
    u, i, sz, vp, ll = ctypes.c_uint, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_longlong
    lib.cuzfp_hip_abi_version.restype = i
    lib.cuzfp_hip_status_string.restype = ctypes.c_char_p
    lib.cuzfp_hip_status_string.argtypes = [i]
    lib.cuzfp_hip_last_hip_error.restype = i
    lib.cuzfp_hip_rate_to_maxbits.restype = u
    lib.cuzfp_hip_rate_to_maxbits.argtypes = [ctypes.c_double, i, u, i]
    lib.cuzfp_hip_stream_bytes.restype = sz
    lib.cuzfp_hip_stream_bytes.argtypes = [i, u, u, u, u]
    lib.cuzfp_hip_maximum_size.restype = sz
    lib.cuzfp_hip_maximum_size.argtypes = [i, u, u, u, u]
    lib.cuzfp_hip_encode.restype = i
    lib.cuzfp_hip_encode.argtypes = [vp, i, u, u, u, ll, ll, ll, u, vp, sz, ctypes.POINTER(sz), vp]
    lib.cuzfp_hip_decode.restype = i
    lib.cuzfp_hip_decode.argtypes = [vp, sz, i, u, u, u, ll, ll, ll, u, vp, vp]
    lib.cuzfp_hip_compress_host.restype = i
    lib.cuzfp_hip_compress_host.argtypes = [vp, i, u, u, u, u, vp, sz, ctypes.POINTER(sz), i]
    lib.cuzfp_hip_decompress_host.restype = i
    lib.cuzfp_hip_decompress_host.argtypes = [vp, sz, i, u, u, u, u, vp, i]
    lib.cuzfp_hip_copy.restype = i
    lib.cuzfp_hip_copy.argtypes = [vp, vp, sz, vp]
    lib.cuzfp_hip_release_host_cache.restype = i
    lib.cuzfp_hip_release_host_cache.argtypes = [i]
    _lib = lib
    return lib


def _check(where: str, rc: int) -> None:
    if rc != 0:
        raise CodecError(where, rc, library().cuzfp_hip_last_hip_error())


def _extents(shape) -> tuple[int, int, int]:
    """(slowest..fastest) shape -> zfp (nx, ny, nz); 0 marks an unused dimension."""
    shape = tuple(int(s) for s in shape)
    if len(shape) == 1:
        return shape[0], 0, 0
    if len(shape) == 2:
        return shape[1], shape[0], 0
    if len(shape) == 3:
        return shape[2], shape[1], shape[0]
    raise ValueError("zfp arrays are 1D, 2D or 3D")


def type_code(dtype) -> int:
    """zfp_type code of a numpy or torch dtype."""
    if hasattr(dtype, "is_floating_point"):  # torch.dtype
        import torch
        dtype = {torch.float32: np.float32, torch.float64: np.float64,
                 torch.int32: np.int32, torch.int64: np.int64}.get(dtype)
        if dtype is None:
            raise TypeError("cuzfp_amd supports float32, float64, int32 and int64")
    return _NP_TYPES[np.dtype(dtype)]


def rate_to_maxbits(rate: float, dtype, dims: int, wra: bool = False) -> int:
    """Bits per block for `rate` bits/value (zfp_stream_set_rate; wra rounds to 64)."""
    return int(library().cuzfp_hip_rate_to_maxbits(float(rate), type_code(dtype), dims, int(wra)))


def stream_bytes(shape, dtype, maxbits: int) -> int:
    nx, ny, nz = _extents(shape)
    n = library().cuzfp_hip_stream_bytes(type_code(dtype), nx, ny, nz, maxbits)
    if n == 0:
        raise CodecError("stream_bytes", 1)
    return int(n)


def maximum_size(shape, dtype, maxbits: int) -> int:
    nx, ny, nz = _extents(shape)
    return int(library().cuzfp_hip_maximum_size(type_code(dtype), nx, ny, nz, maxbits))


def _stream_handle(stream):
    import torch
    if stream is None:
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream)


def _strides(x):
    """Element strides (sx, sy, sz) of a torch tensor in zfp order."""
    st = list(x.stride())[::-1] + [0, 0]
    return st[0], st[1] if x.dim() > 1 else 0, st[2] if x.dim() > 2 else 0


def _broadcast(x) -> bool:
    """True for a view with a zero stride on an axis of extent > 1 (expand /
    broadcast): the C-ABI reads a zero stride as "contiguous default", so such
    a view must not be passed through as it is."""
    return any(st == 0 and n > 1 for st, n in zip(x.stride(), x.shape))


def _check_host_out(out: np.ndarray, shape, dtype, what: str) -> None:
    if not isinstance(out, np.ndarray) or not out.flags.c_contiguous:
        raise ValueError(f"{what}: out must be a C-contiguous numpy array")
    if out.dtype != np.dtype(dtype):
        raise ValueError(f"{what}: out has dtype {out.dtype}, expected {np.dtype(dtype)}")
    if shape is not None and tuple(out.shape) != tuple(int(s) for s in shape):
        raise ValueError(f"{what}: out has shape {out.shape}, expected {tuple(shape)}")


def encode(x, maxbits: int, out=None, stream=None):
    """Compress a CUDA tensor; returns the stream as an int64 tensor of 64-bit words.

    Bit-exact with zfp 0.5.0 fixed-rate mode (``zfp_compress`` with
    minbits = maxbits).  Asynchronous on `stream` (default: torch's current).
    """
    import torch
    if not x.is_cuda:
        raise ValueError("encode: expects a device tensor (use compress_host for host arrays)")
    if _broadcast(x):
        # materialise a broadcast view (a zero stride means "contiguous" to the
        # C-ABI) on the launch stream, after the work already queued on torch's
        # current stream.  The copy is allocated on that stream, so the kernel
        # that reads it is ordered before any reuse; the broadcast source was
        # allocated on the current stream and is read on s, so it is recorded
        # there (the caching allocator then waits for s before reusing it).
        cur = torch.cuda.current_stream(x.device)
        s = cur if stream is None else stream
        s.wait_stream(cur)
        src = x
        with torch.cuda.stream(s):
            x = src.contiguous()
        if s != cur:
            src.record_stream(s)
    t = type_code(x.dtype)
    nx, ny, nz = _extents(x.shape)
    nbytes = stream_bytes(x.shape, x.dtype, maxbits)
    if out is None:
        out = torch.empty(nbytes // 8, dtype=torch.int64, device=x.device)
    sx, sy, sz = _strides(x)
    got = ctypes.c_size_t(0)
    rc = library().cuzfp_hip_encode(x.data_ptr(), t, nx, ny, nz, sx, sy, sz, maxbits,
                                    out.data_ptr(), out.numel() * out.element_size(),
                                    ctypes.byref(got), _stream_handle(stream))
    _check("encode", rc)
    return out


def decode(words, shape, dtype, maxbits: int, out=None, stream=None):
    """Decompress a device stream (int64 words) into a new (or given) CUDA tensor."""
    import torch
    if not words.is_cuda:
        raise ValueError("decode: expects a device stream")
    if out is None:
        out = torch.empty(tuple(shape), dtype=dtype, device=words.device)
    elif _broadcast(out):
        raise ValueError("decode: out is a broadcast view (zero stride); its elements alias each other")
    t = type_code(out.dtype)
    nx, ny, nz = _extents(out.shape)
    sx, sy, sz = _strides(out)
    rc = library().cuzfp_hip_decode(words.data_ptr(), words.numel() * words.element_size(), t,
                                    nx, ny, nz, sx, sy, sz, maxbits, out.data_ptr(),
                                    _stream_handle(stream))
    _check("decode", rc)
    return out


def copy(src, dst, stream=None):
    """Device-to-device copy through cuzfp_hip_copy (16-byte non-temporal
    accesses): the bandwidth calibrator bench.py reports beside the codec."""
    for name, t in (("src", src), ("dst", dst)):
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError(f"copy: {name} must be a contiguous device tensor")
    nbytes = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() < nbytes:
        raise ValueError("copy: destination too small")
    _check("copy", library().cuzfp_hip_copy(src.data_ptr(), dst.data_ptr(), nbytes, _stream_handle(stream)))
    return dst


def compress_host(a: np.ndarray, maxbits: int, nstreams: int = 4, out: np.ndarray | None = None):
    """Host array -> host stream (uint64 words) through the pinned, overlapped pipeline."""
    a = np.ascontiguousarray(a)
    nx, ny, nz = _extents(a.shape)
    nbytes = stream_bytes(a.shape, a.dtype, maxbits)
    if out is None:
        out = np.empty(nbytes // 8, dtype=np.uint64)
    else:
        _check_host_out(out, None, out.dtype, "compress_host")
        if out.nbytes < nbytes:
            raise ValueError(f"compress_host: out holds {out.nbytes} bytes, the stream needs {nbytes}")
    got = ctypes.c_size_t(0)
    rc = library().cuzfp_hip_compress_host(a.ctypes.data, type_code(a.dtype), nx, ny, nz, maxbits,
                                           out.ctypes.data, out.nbytes, ctypes.byref(got), nstreams)
    _check("compress_host", rc)
    return out


def release_host_cache(device: int = -1) -> None:
    """Free the host pipeline's retained device buffers, pinned staging buffers,
    streams and events (cuzfp_hip_release_host_cache; -1 = the current device)."""
    _check("release_host_cache", library().cuzfp_hip_release_host_cache(device))


def decompress_host(words: np.ndarray, shape, dtype, maxbits: int, nstreams: int = 4,
                    out: np.ndarray | None = None):
    words = np.ascontiguousarray(words)
    if out is None:
        out = np.empty(tuple(shape), dtype=dtype)
    else:
        _check_host_out(out, shape, dtype, "decompress_host")
    nx, ny, nz = _extents(out.shape)
    rc = library().cuzfp_hip_decompress_host(words.ctypes.data, words.nbytes, type_code(out.dtype),
                                             nx, ny, nz, maxbits, out.ctypes.data, nstreams)
    _check("decompress_host", rc)
    return out
