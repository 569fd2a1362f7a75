"""GPU parity: the HIP codec (through the C-ABI) against the CPU oracle.

Bar: compressed streams bit-exact with zfp 0.5.0 fixed-rate
mode, decompressed arrays bit-exact with zfp 0.5.0's decoder.  Cases follow the
reference's own tests -- the sanity ramps (src/tests/t_sanity_check_{1,2,3}.cpp),
the differential fuzz space of src/utils/test.py:101-132 (random dims, rates
1..31, f32/f64) -- plus partial blocks, strides, integer fields and
denormal / zero / huge-range blocks.
"""
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
    assert np.array_equal(words, restatement.compress(a, mb))
    assert np.array_equal(y.astype(np.int64), a.astype(np.int64))


@pytest.mark.parametrize("dims", [1, 2, 3])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("kind", ["normal", "smooth", "range", "sparse"])
def test_fuzz_vs_oracle(dims, dtype, kind, cuda, restatement):
    rng = np.random.default_rng(hash((dims, np.dtype(dtype).str, kind)) & 0xffffffff)
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
