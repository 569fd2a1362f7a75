"""Launch the 3D codec kernels a few times for profiler runs (rocprofv3 --pmc).

    rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU ... -- python tools/kernel_probe.py [--field F] [--reps R]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cuzfp_amd as cz  # noqa: E402
from cuzfp_amd.datagen import polynomial_field, splitmix_uniform  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--field", default="polynomial")
p.add_argument("--dtype", default="float32")
p.add_argument("--rate", type=float, default=8)
p.add_argument("--size", type=int, default=256)
p.add_argument("--dims", type=int, default=3, choices=[1, 2, 3])
p.add_argument("--reps", type=int, default=5)
a = p.parse_args()
shape = (a.size,) * a.dims
arr = polynomial_field(shape, a.dtype) if a.field == "polynomial" else splitmix_uniform(shape, a.dtype)
x = torch.from_numpy(arr).cuda()
mb = cz.rate_to_maxbits(a.rate, arr.dtype, a.dims)
w = cz.encode(x, mb)
y = cz.decode(w, shape, x.dtype, mb)
for _ in range(a.reps):
    cz.encode(x, mb, out=w)
for _ in range(a.reps):
    cz.decode(w, shape, x.dtype, mb, out=y)
torch.cuda.synchronize()
print("ok")
