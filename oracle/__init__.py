"""TEST INFRASTRUCTURE ONLY -- CPU checkers for the HIP zfp codec.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package.  The shipped codec (``cuzfp_amd``) never does.

Two checkers with one Python surface:

* :data:`restatement` -- ``oracle/liboracle.so``, our plain-C restatement of the
  zfp 0.5.0 fixed-rate codec (``oracle/zfp_oracle.c``).
* :data:`reference` -- ``oracle/_ref/libzfp_ref.so``, the reference's vendored
  CPU zfp 0.5.0 (``/root/reference/src/thirdparty_builtin/zfp-0.5.0``) compiled
  by ``oracle/Makefile``; ``None`` when it has not been built.

Type codes follow ``src/cuZFP/zfp_structs.h:46-52``: 1 int32, 2 int64,
3 float, 4 double.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
TYPE_CODES = {np.dtype(np.int32): 1, np.dtype(np.int64): 2,
              np.dtype(np.float32): 3, np.dtype(np.float64): 4}

_u = ctypes.c_uint
_i = ctypes.c_int
_sz = ctypes.c_size_t
_vp = ctypes.c_void_p


def build(with_reference: bool | None = None) -> None:
    """Compile the restatement (always) and the reference (when its sources exist)."""
    targets = ["oracle"]
    if with_reference is None:
        with_reference = os.path.isdir("/root/reference/src/thirdparty_builtin/zfp-0.5.0")
    if with_reference:
        targets.append("ref")
    subprocess.check_call(["make", "-s", "-C", HERE] + targets)


def _shape_args(shape):
    """numpy shape (C order, slowest first) -> zfp (nx, ny, nz)."""
    dims = len(shape)
    if dims == 1:
        return shape[0], 0, 0
    if dims == 2:
        return shape[1], shape[0], 0
    if dims == 3:
        return shape[2], shape[1], shape[0]
    raise ValueError("zfp arrays are 1D, 2D or 3D")


class _Codec:
    """Common numpy front end over a C codec library."""

    def __init__(self, lib: ctypes.CDLL, kind: str):
        self.lib = lib
        self.kind = kind

    # -- stream sizing --------------------------------------------------------
    @staticmethod
    def blocks(shape) -> int:
        n = 1
        for s in shape:
            n *= (s + 3) // 4
        return n

    @classmethod
    def stream_bytes(cls, shape, maxbits: int) -> int:
        return ((cls.blocks(shape) * maxbits + 63) // 64) * 8

    # -- codec ----------------------------------------------------------------
    def compress(self, a: np.ndarray, maxbits: int, strides=(0, 0, 0)) -> np.ndarray:
        a = np.asarray(a)
        if not strides or strides == (0, 0, 0):
            a = np.ascontiguousarray(a)
        nx, ny, nz = _shape_args(a.shape)
        t = TYPE_CODES[a.dtype]
        cap = self.stream_bytes(a.shape, maxbits) + 64
        out = np.zeros(cap // 8, dtype=np.uint64)
        n = self._compress(t, nx, ny, nz, strides, maxbits, a, out, cap)
        if n == 0:
            raise ValueError(f"{self.kind}: compress rejected its arguments")
        return out[: n // 8].copy()

    def decompress(self, stream: np.ndarray, shape, dtype, maxbits: int) -> np.ndarray:
        dtype = np.dtype(dtype)
        stream = np.ascontiguousarray(stream, dtype=np.uint64)
        nx, ny, nz = _shape_args(tuple(shape))
        out = np.zeros(shape, dtype=dtype)
        ok = self._decompress(TYPE_CODES[dtype], nx, ny, nz, (0, 0, 0), maxbits,
                              stream, stream.nbytes, out)
        if not ok:
            raise ValueError(f"{self.kind}: decompress rejected its arguments")
        return out


class Restatement(_Codec):
    def __init__(self, path: str):
        lib = ctypes.CDLL(path)
        for name in ("oracle_compress", "oracle_compress_int"):
            f = getattr(lib, name)
            f.restype = _sz
            f.argtypes = [_i, _u, _u, _u, _i, _i, _i, _u, _vp, _vp, _sz]
        for name in ("oracle_decompress", "oracle_decompress_int"):
            f = getattr(lib, name)
            f.restype = _i
            f.argtypes = [_i, _u, _u, _u, _i, _i, _i, _u, _vp, _sz, _vp]
        lib.oracle_jenkins_hash.restype = ctypes.c_uint32
        lib.oracle_jenkins_hash.argtypes = [_vp, _sz]
        lib.oracle_rate_to_maxbits.restype = _u
        lib.oracle_rate_to_maxbits.argtypes = [ctypes.c_double, _i, _u, _i]
        super().__init__(lib, "restatement")

    def rate_to_maxbits(self, rate: float, dtype, dims: int, wra: bool = False) -> int:
        return self.lib.oracle_rate_to_maxbits(rate, TYPE_CODES[np.dtype(dtype)], dims, int(wra))

    def jenkins_hash(self, a: np.ndarray) -> int:
        """testzfp's array checksum (testzfp.cpp:74-89)."""
        a = np.ascontiguousarray(a)
        return int(self.lib.oracle_jenkins_hash(a.ctypes.data, a.nbytes))

    def _compress(self, t, nx, ny, nz, st, maxbits, a, out, cap):
        f = self.lib.oracle_compress if t >= 3 else self.lib.oracle_compress_int
        return f(t, nx, ny, nz, st[0], st[1], st[2], maxbits, a.ctypes.data, out.ctypes.data, cap)

    def _decompress(self, t, nx, ny, nz, st, maxbits, stream, nbytes, out):
        f = self.lib.oracle_decompress if t >= 3 else self.lib.oracle_decompress_int
        return f(t, nx, ny, nz, st[0], st[1], st[2], maxbits, stream.ctypes.data, nbytes,
                 out.ctypes.data)


class Reference(_Codec):
    """The reference's own CPU zfp 0.5.0 (float/double arrays; int blocks)."""

    def __init__(self, path: str):
        lib = ctypes.CDLL(path)
        lib.ref_compress.restype = _sz
        lib.ref_compress.argtypes = [_i, _u, _u, _u, _i, _i, _i, _u, _vp, _vp, _sz]
        lib.ref_decompress.restype = _i
        lib.ref_decompress.argtypes = [_i, _u, _u, _u, _i, _i, _i, _u, _vp, _sz, _vp]
        lib.ref_rate_to_maxbits.restype = _u
        lib.ref_rate_to_maxbits.argtypes = [ctypes.c_double, _i, _u, _i]
        lib.ref_encode_int_blocks.restype = _sz
        lib.ref_encode_int_blocks.argtypes = [_i, _u, _u, _sz, _vp, _vp, _sz]
        lib.ref_decode_int_blocks.restype = _i
        lib.ref_decode_int_blocks.argtypes = [_i, _u, _u, _sz, _vp, _sz, _vp]
        lib.ref_time_roundtrip.restype = ctypes.c_double
        lib.ref_time_roundtrip.argtypes = [_i, _u, _u, _u, _u, _vp, _vp, _i, _i,
                                           ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_double)]
        super().__init__(lib, "reference")

    def rate_to_maxbits(self, rate: float, dtype, dims: int, wra: bool = False) -> int:
        return self.lib.ref_rate_to_maxbits(rate, TYPE_CODES[np.dtype(dtype)], dims, int(wra))

    def _compress(self, t, nx, ny, nz, st, maxbits, a, out, cap):
        if t < 3:
            raise ValueError("zfp 0.5.0 zfp_compress rejects integer fields (zfp.c:618-624)")
        return self.lib.ref_compress(t, nx, ny, nz, st[0], st[1], st[2], maxbits,
                                     a.ctypes.data, out.ctypes.data, cap)

    def _decompress(self, t, nx, ny, nz, st, maxbits, stream, nbytes, out):
        return self.lib.ref_decompress(t, nx, ny, nz, st[0], st[1], st[2], maxbits,
                                       stream.ctypes.data, nbytes, out.ctypes.data)

    def encode_int_blocks(self, blocks: np.ndarray, dims: int, maxbits: int) -> np.ndarray:
        """Contiguous 4^dims integer blocks through zfp_encode_block_int{32,64}_{dims}."""
        blocks = np.ascontiguousarray(blocks)
        nb = blocks.size >> (2 * dims)
        cap = ((nb * maxbits + 63) // 64) * 8 + 64
        out = np.zeros(cap // 8, dtype=np.uint64)
        n = self.lib.ref_encode_int_blocks(TYPE_CODES[blocks.dtype], dims, maxbits, nb,
                                           blocks.ctypes.data, out.ctypes.data, cap)
        return out[: n // 8].copy()

    def decode_int_blocks(self, stream, dims: int, maxbits: int, nblocks: int, dtype) -> np.ndarray:
        dtype = np.dtype(dtype)
        stream = np.ascontiguousarray(stream, dtype=np.uint64)
        out = np.zeros(nblocks << (2 * dims), dtype=dtype)
        self.lib.ref_decode_int_blocks(TYPE_CODES[dtype], dims, maxbits, nblocks,
                                       stream.ctypes.data, stream.nbytes, out.ctypes.data)
        return out

    def time_roundtrip(self, a: np.ndarray, maxbits: int, threads: int = 1, reps: int = 3):
        """Median (round trip, encode, decode) seconds of zfp_compress+zfp_decompress."""
        a = np.ascontiguousarray(a)
        out = np.empty_like(a)
        nx, ny, nz = _shape_args(a.shape)
        e, d = ctypes.c_double(), ctypes.c_double()
        rt = self.lib.ref_time_roundtrip(TYPE_CODES[a.dtype], nx, ny, nz, maxbits,
                                         a.ctypes.data, out.ctypes.data, threads, reps,
                                         ctypes.byref(e), ctypes.byref(d))
        return rt, e.value, d.value, out


def _load(cls, path):
    return cls(path) if os.path.exists(path) else None


restatement = _load(Restatement, os.path.join(HERE, "liboracle.so"))
reference = _load(Reference, os.path.join(HERE, "_ref", "libzfp_ref.so"))


def reload() -> None:
    """Re-open the libraries after :func:`build`."""
    global restatement, reference
    restatement = _load(Restatement, os.path.join(HERE, "liboracle.so"))
    reference = _load(Reference, os.path.join(HERE, "_ref", "libzfp_ref.so"))
