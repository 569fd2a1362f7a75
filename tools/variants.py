"""Build and time compile-time variants of the codec library (design tool).

  python tools/variants.py build NAME "-DFLAG=1 ..." [NAME "FLAGS" ...]   # here
  python tools/variants.py run [--size S] [--field F] NAME [NAME ...]      # GPU box

Each variant is a full libcuzfp_hip.so under build/var/NAME, loaded through
CUZFP_HIP_LIB in a child process; run prints encode/decode microseconds of the
3D float32 rate-8 kernels per variant.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "build", "var")
UNITS = ("inst_f32", "inst_f64", "inst_i32", "inst_i64", "capi")


def build(pairs):
    from cuzfp_amd import build as b
    procs = []
    for name, flags in pairs:
        d = os.path.join(OUT, name)
        os.makedirs(d, exist_ok=True)
        for u in UNITS:
            procs.append(subprocess.Popen([b.HIPCC, *b.CXXFLAGS, *flags.split(), "-c",
                                           os.path.join(b.CSRC, u + ".hip"), "-o", os.path.join(d, u + ".o")]))
    assert all(p.wait() == 0 for p in procs)
    for name, _ in pairs:
        d = os.path.join(OUT, name)
        subprocess.check_call([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o",
                               os.path.join(d, "libcuzfp_hip.so"), *[os.path.join(d, u + ".o") for u in UNITS]])
        for u in UNITS:
            os.remove(os.path.join(d, u + ".o"))
    print("built", [n for n, _ in pairs])


CODE = """
import os, sys, json, torch
sys.path.insert(0, {root!r})
os.environ['CUZFP_HIP_LIB'] = {lib!r}
import cuzfp_amd as cz
from cuzfp_amd.datagen import polynomial_field, splitmix_uniform
shape = ({size},)*3
arr = polynomial_field(shape, {dtype!r}) if {field!r} == 'polynomial' else splitmix_uniform(shape, {dtype!r})
x = torch.from_numpy(arr).cuda()
mb = cz.rate_to_maxbits({rate}, arr.dtype, 3)
w = cz.encode(x, mb); y = cz.decode(w, shape, x.dtype, mb)
def t(fn):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20): fn()
    g.replay(); torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    r = []
    for _ in range(11):  # median of 11 batches of 2 x 20 (hipGraph replays)
        torch.cuda.synchronize(); e0.record()
        g.replay(); g.replay()
        e1.record(); torch.cuda.synchronize()
        r.append(e0.elapsed_time(e1) / 40 * 1000)
    return round(sorted(r)[5], 2)
def step():
    cz.encode(x, mb, out=w); cz.decode(w, shape, x.dtype, mb, out=y)
print(json.dumps(dict(enc_us=t(lambda: cz.encode(x, mb, out=w)), dec_us=t(lambda: cz.decode(w, shape, x.dtype, mb, out=y)), step_us=t(step))))
"""


def run(names, size, field, dtype="float32", rate=8):
    for name in names:
        lib = os.path.join(OUT, name, "libcuzfp_hip.so")
        code = CODE.format(root=ROOT, lib=lib, size=size, field=field, dtype=dtype, rate=rate)
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
        if r.returncode:
            print(name, "FAILED", r.stderr[-500:])
            sys.exit(r.returncode)
        print(f"{name:12s} {field:10s} {size} {r.stdout.strip()}", flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        a = sys.argv[2:]
        build(list(zip(a[0::2], a[1::2])))
    else:
        import argparse
        p = argparse.ArgumentParser()
        p.add_argument("cmd")
        p.add_argument("--size", type=int, default=256)
        p.add_argument("--field", default="polynomial")
        p.add_argument("--dtype", default="float32")
        p.add_argument("--rate", type=int, default=8)
        p.add_argument("names", nargs="+")
        a = p.parse_args()
        run(a.names, a.size, a.field, a.dtype, a.rate)
