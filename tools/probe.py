"""Phase-cost probes of the 3D f32 codec kernels (design tool, not a test).

  python tools/probe.py build            # here: compile build/probe/p{0,1,2}/libcuzfp_hip.so
  python tools/probe.py run [--size S]   # GPU box: time encode/decode of each variant

Variants (CUZFP_PROBE in zfp_block.hpp): p0 = the product kernels, p1 = no
embedded plane coder (planes still transposed), p2 = no transpose either.  The
outputs of p1/p2 are meaningless; only their kernel times are read.
"""
from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "build", "probe")


def build():
    from cuzfp_amd import build as b
    procs = []
    for v in (0, 1, 2):
        d = os.path.join(OUT, f"p{v}")
        os.makedirs(d, exist_ok=True)
        objs = []
        for u in ("inst_f32", "inst_f64", "inst_i32", "inst_i64", "capi"):
            o = os.path.join(d, u + ".o")
            objs.append(o)
            procs.append(subprocess.Popen([b.HIPCC, *b.CXXFLAGS, f"-DCUZFP_PROBE={v}", "-c",
                                           os.path.join(b.CSRC, u + ".hip"), "-o", o]))
    assert all(p.wait() == 0 for p in procs)
    for v in (0, 1, 2):
        d = os.path.join(OUT, f"p{v}")
        objs = [os.path.join(d, u + ".o") for u in ("inst_f32", "inst_f64", "inst_i32", "inst_i64", "capi")]
        subprocess.check_call([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o",
                               os.path.join(d, "libcuzfp_hip.so"), *objs])
    print("built", OUT)


def run(size, field, reps=20):
    res = {}
    for v in (0, 1, 2):
        lib = os.path.join(OUT, f"p{v}", "libcuzfp_hip.so")
        code = f"""
import os, sys, json, torch, numpy as np
sys.path.insert(0, {ROOT!r})
os.environ['CUZFP_HIP_LIB'] = {lib!r}
import cuzfp_amd as cz
from cuzfp_amd.datagen import polynomial_field, splitmix_uniform
shape = ({size},)*3
arr = polynomial_field(shape) if {field!r} == 'polynomial' else splitmix_uniform(shape)
x = torch.from_numpy(arr).cuda()
mb = cz.rate_to_maxbits(8, arr.dtype, 3)
w = cz.encode(x, mb); y = cz.decode(w, shape, x.dtype, mb)
def t(fn):
    for _ in range(3): fn()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record()
    for _ in range({reps}): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / {reps} * 1000
print(json.dumps(dict(enc_us=t(lambda: cz.encode(x, mb, out=w)), dec_us=t(lambda: cz.decode(w, shape, x.dtype, mb, out=y)))))
"""
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
        if r.returncode:
            print(r.stderr[-2000:])
            raise SystemExit(r.returncode)
        res[f"p{v}"] = r.stdout.strip().splitlines()[-1]
        print(f"p{v}", res[f"p{v}"], flush=True)


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--field", default="polynomial")
    a = ap.parse_args()
    if a.cmd == "build":
        build()
    else:
        run(a.size, a.field)
