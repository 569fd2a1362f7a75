"""Deterministic synthetic fields (the reference's data generators, IEEE-reproducible).

* :func:`polynomial_field` -- testzfp's separable field
  ``f(x) = x - 3x^2 + 4x^4`` at ``x = (2i - n + 1)/n``, the input of zfp 0.5.0's
  regression test (zfp-0.5.0/tests/testzfp.cpp:33-72).  Each operation is a
  separate IEEE op in the array's precision, like the reference's ``volatile``
  temporaries, so the result is bit-identical to testzfp's and is pinned by its
  Jenkins checksums (testzfp.cpp:475-489) in tests/test_oracle.py.
* :func:`splitmix_uniform` -- uniform values in [-1, 1) from the splitmix64
  integer generator; rough data that keeps every bit plane busy (the
  worst case for the plane coder).
* :func:`ramp` -- ``f[i] = i``, the input of the reference's sanity tests
  (src/tests/t_sanity_check_{1,2,3}.cpp).
* :func:`sine_field` -- ``f[x] = (T)(sin(x * 3.14/180) * 10)``, the input of
  the reference's 1D encode/decode test (src/tests/t_encode_decode_1.cpp:15-30),
  BASELINE.json configs[0] at 1M values.

Shapes are numpy order (slowest first).
"""
from __future__ import annotations

import numpy as np


def _poly(x):
    xx = x * x
    yy = xx * x.dtype.type(4) - x.dtype.type(3)
    return x + xx * yy


def _axis(n, dtype):
    dt = np.dtype(dtype).type
    i = np.arange(n, dtype=np.int64)
    x = (2 * i - n + 1).astype(dtype) / dt(n)
    return _poly(x) if n > 1 else np.ones(n, dtype=dtype)


def polynomial_field(shape, dtype=np.float32) -> np.ndarray:
    """testzfp.cpp:46-72 ``initialize(p, nx, ny, nz, polynomial)``: fx * fy * fz."""
    dtype = np.dtype(dtype)
    shape = tuple(int(s) for s in shape)
    axes = [_axis(n, dtype) for n in shape[::-1]]  # fx, fy, fz
    # the reference multiplies fx * fy * fz left to right, with 1 for an
    # absent dimension: (fx * fy) * fz
    f = axes[0]
    if len(shape) >= 2:
        f = axes[0][None, :] * axes[1][:, None]
    if len(shape) == 3:
        f = f[None, :, :] * axes[2][:, None, None]
    return np.ascontiguousarray(f.astype(dtype, copy=False))


def polynomial_slab(global_shape, z0: int, z1: int, dtype=np.float32) -> np.ndarray:
    """Planes [z0, z1) of polynomial_field(global_shape) (3D), built per slab so a
    rank never materialises the global array."""
    dtype = np.dtype(dtype)
    nz, ny, nx = (int(s) for s in global_shape)
    fx, fy, fz = _axis(nx, dtype), _axis(ny, dtype), _axis(nz, dtype)[z0:z1]
    f = (fx[None, :] * fy[:, None])[None, :, :] * fz[:, None, None]
    return np.ascontiguousarray(f.astype(dtype, copy=False))


def polynomial_slab_device(gshape, z0: int, z1: int, device):
    """datagen.polynomial_slab built on the GPU: the three 1D axes come from the
    CPU generator (testzfp's IEEE op order) and the two products are exact-
    rounded f32 multiplies on the device, so the slab is bit-identical (the
    stream hash against the reference's checks it)."""
    import torch
    nz, ny, nx = gshape
    fx = torch.from_numpy(_axis(nx, np.float32)).to(device)
    fy = torch.from_numpy(_axis(ny, np.float32)).to(device)
    fz = torch.from_numpy(_axis(nz, np.float32)[z0:z1].copy()).to(device)
    return ((fx[None, :] * fy[:, None])[None, :, :] * fz[:, None, None]).contiguous()


def splitmix64(n: int, seed: int = 42) -> np.ndarray:
    """n successive outputs of splitmix64 seeded with `seed`."""
    with np.errstate(over="ignore"):
        idx = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed) + idx * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def splitmix_uniform(shape, dtype=np.float32, seed: int = 42) -> np.ndarray:
    """Uniform values in [-1, 1): top 53 (f64) / 24 (f32) bits of splitmix64."""
    dtype = np.dtype(dtype)
    n = int(np.prod(shape))
    z = splitmix64(n, seed)
    if dtype == np.float32:
        u = (z >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -23) - np.float32(1)
    else:
        u = (z >> np.uint64(11)).astype(np.float64) * (2.0 ** -52) - 1.0
    return u.astype(dtype).reshape(shape)


def ramp(shape, dtype=np.float32) -> np.ndarray:
    return np.arange(int(np.prod(shape)), dtype=dtype).reshape(shape)


def sine_field(n: int, dtype=np.float32) -> np.ndarray:
    """src/tests/t_encode_decode_1.cpp:18-23: v = x * (3.14/180.) in double,
    value = (T)(sin(v) * 10.)."""
    v = np.arange(n, dtype=np.float64) * (3.14 / 180.0)
    return (np.sin(v) * 10.0).astype(dtype)
