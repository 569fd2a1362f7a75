"""GPU parity of cuzfp_hip_decode_encode: one launch that decodes one stream and
encodes another array must give exactly what cuzfp_hip_decode and
cuzfp_hip_encode give (the combined kernel runs the same per-lane codec bodies;
the round-trip chain below also checks the stream against the CPU
restatement of zfp 0.5.0), and must refuse what it does not cover.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import cuzfp_amd as cz
from cuzfp_amd.datagen import polynomial_field, splitmix_uniform


@pytest.mark.parametrize("shape", [(64, 64, 64), (16, 16, 256), (8, 12, 20), (4, 4, 4)])
@pytest.mark.parametrize("rate", [8, 16, 4])
def test_decode_encode_matches_separate_calls(cuda, restatement, shape, rate):
    import torch
    mb = cz.rate_to_maxbits(rate, np.float32, 3, wra=True)
    a = polynomial_field(shape)
    b = splitmix_uniform(shape, seed=7)
    xa = torch.from_numpy(a).to(cuda)
    xb = torch.from_numpy(b).to(cuda)
    wa = cz.encode(xa, mb)                       # the stream to decode
    wb_ref = cz.encode(xb, mb)                   # what encoding b gives
    ya_ref = cz.decode(wa, shape, torch.float32, mb)
    ya = torch.full_like(xa, float("nan"))
    wb = torch.full_like(wb_ref, -1)
    cz.decode_encode(wa, ya, xb, wb, mb)
    torch.cuda.synchronize()
    assert torch.equal(wb, wb_ref)
    assert torch.equal(ya, ya_ref)
    if np.prod(shape) <= 64 ** 3:
        ref = restatement.compress(b, mb)
        assert np.array_equal(wb.cpu().numpy().view(np.uint64), ref)
        assert np.array_equal(ya.cpu().numpy(),
                              restatement.decompress(wa.cpu().numpy().view(np.uint64), shape, np.float32, mb))


def test_decode_encode_chain(cuda):
    """Round trips pipelined through the combined launch (encode 0; decode k with
    encode k+1; decode last) over two stream buffers and distinct fields:
    every stream and every decoded field equals the separate calls'."""
    import torch
    shape, mb = (32, 64, 64), 512
    xs = [torch.from_numpy(splitmix_uniform(shape, seed=s)).to(cuda) for s in range(5)]
    refs = [cz.encode(x, mb) for x in xs]
    decs = [cz.decode(w, shape, torch.float32, mb) for w in refs]
    w = [torch.empty_like(refs[0]), torch.empty_like(refs[0])]
    ys = [torch.empty_like(xs[0]) for _ in xs]
    cz.encode(xs[0], mb, out=w[0])
    for k in range(len(xs) - 1):
        cz.decode_encode(w[k & 1], ys[k], xs[k + 1], w[(k + 1) & 1], mb)
        torch.cuda.synchronize()
        assert torch.equal(w[(k + 1) & 1], refs[k + 1])
        assert torch.equal(ys[k], decs[k])
    cz.decode(w[(len(xs) - 1) & 1], shape, torch.float32, mb, out=ys[-1])
    torch.cuda.synchronize()
    assert torch.equal(ys[-1], decs[-1])


@pytest.mark.parametrize("case", ["f64", "2d", "maxbits480", "ragged"])
def test_decode_encode_refuses(cuda, case):
    import torch
    dtype = torch.float64 if case == "f64" else torch.float32
    shape = {"2d": (64, 64), "ragged": (6, 8, 8)}.get(case, (8, 8, 8))
    mb = 480 if case == "maxbits480" else 512
    x = torch.zeros(shape, dtype=dtype, device=cuda)
    y = torch.empty_like(x)
    w_in = cz.encode(x, mb)
    w_out = torch.empty_like(w_in)
    with pytest.raises(cz.CodecError) as e:
        cz.decode_encode(w_in, y, x, w_out, mb)
    assert e.value.status == 2  # unsupported: the caller makes the two calls
