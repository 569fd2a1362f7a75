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


VARIANTS = (0, 1, 2, 9)


def build(variants=VARIANTS):
    from cuzfp_amd import build as b
    procs = []
    for v in variants:
        d = os.path.join(OUT, f"p{v}")
        os.makedirs(d, exist_ok=True)
        objs = []
        for u in ("inst_f32", "inst_f64", "inst_i32", "inst_i64", "capi"):
            o = os.path.join(d, u + ".o")
            objs.append(o)
            procs.append(subprocess.Popen([b.HIPCC, *b.CXXFLAGS, f"-DCUZFP_PROBE={v}", "-c",
                                           os.path.join(b.CSRC, u + ".hip"), "-o", o]))
    import time
    t0 = time.time()
    while any(p.poll() is None for p in procs):  # a heartbeat line for long builds
        time.sleep(2)
        if int(time.time() - t0) % 30 < 2:
            print(f"building ... {int(time.time() - t0)} s", flush=True)
    assert all(p.returncode == 0 for p in procs)
    for v in variants:
        d = os.path.join(OUT, f"p{v}")
        objs = [os.path.join(d, u + ".o") for u in ("inst_f32", "inst_f64", "inst_i32", "inst_i64", "capi")]
        subprocess.check_call([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o",
                               os.path.join(d, "libcuzfp_hip.so"), *objs])
    print("built", OUT)


def _shape(size, dims):
    return "(" + ",".join([str(size)] * dims) + ",)"


def run(size, field, dims=3, rate=8.0, reps=20, dtype="float32"):
    res = {}
    for v in (0, 1, 2):
        lib = os.path.join(OUT, f"p{v}", "libcuzfp_hip.so")
        code = f"""
import os, sys, json, torch, numpy as np
sys.path.insert(0, {ROOT!r})
os.environ['CUZFP_HIP_LIB'] = {lib!r}
import cuzfp_amd as cz
from cuzfp_amd.datagen import polynomial_field, splitmix_uniform
shape = {_shape(size, dims)}
arr = polynomial_field(shape, {dtype!r}) if {field!r} == 'polynomial' else splitmix_uniform(shape, {dtype!r})
x = torch.from_numpy(arr).cuda()
mb = cz.rate_to_maxbits({rate}, arr.dtype, {dims})
w = cz.encode(x, mb); y = cz.decode(w, shape, x.dtype, mb)
def t(fn):  # a hipGraph of {reps} launches, median of 11 replays (eager launches can be host-bound)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range({reps}): fn()
    g.replay(); torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    r = []
    for _ in range(11):
        torch.cuda.synchronize(); e0.record()
        g.replay()
        e1.record(); torch.cuda.synchronize()
        r.append(e0.elapsed_time(e1) / {reps} * 1000)
    return sorted(r)[5]
print(json.dumps(dict(enc_us=t(lambda: cz.encode(x, mb, out=w)), dec_us=t(lambda: cz.decode(w, shape, x.dtype, mb, out=y)))))
"""
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
        if r.returncode:
            print(r.stderr[-2000:])
            raise SystemExit(r.returncode)
        res[f"p{v}"] = r.stdout.strip().splitlines()[-1]
        print(f"p{v}", res[f"p{v}"], flush=True)


STAMP_CODE = r"""
import os, sys, json, ctypes, torch, numpy as np
sys.path.insert(0, @ROOT@)
os.environ['CUZFP_HIP_LIB'] = @LIB@
import cuzfp_amd as cz
from cuzfp_amd.datagen import polynomial_field, splitmix_uniform
shape = @SHAPE@
arr = polynomial_field(shape, @DTYPE@) if @FIELD@ == 'polynomial' else splitmix_uniform(shape, @DTYPE@)
x = torch.from_numpy(arr).cuda()
mb = cz.rate_to_maxbits(@RATE@, arr.dtype, @DIMS@)
lib = cz.library()
w = cz.encode(x, mb); y = cz.decode(w, shape, x.dtype, mb)
nw = min((@SIZE@ // 4) ** @DIMS@ // 64, 65536)
out = {}
for name, fn in (("encode", lambda: cz.encode(x, mb, out=w)), ("decode", lambda: cz.decode(w, shape, x.dtype, mb, out=y))):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    sfx = "_f64" if @DTYPE@ == "float64" else ""  # each unit has its own stamp buffer
    getattr(lib, "cuzfp_hip_probe_clear" + sfx)()
    # back to back, as in the bench: the second launch's stamps overwrite the first's
    for _ in range(@BACK@): fn()
    torch.cuda.synchronize()
    buf = np.zeros(65536 * 10, np.uint64)
    getattr(lib, "cuzfp_hip_probe_stamps" + sfx)(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes))
    np.save(os.path.join(@OUTDIR@, "stamps_" + name + "_" + @FIELD@ + "_" + str(@SIZE@) + ".npy"), buf.reshape(-1, 10)[:nw])
print("ok")
"""


def stamps(size, field, outdir, back=1, dims=3, rate=8.0, dtype="float32", variant="p9"):
    lib = os.path.join(OUT, variant, "libcuzfp_hip.so")
    code = STAMP_CODE.replace("@ROOT@", repr(ROOT)).replace("@LIB@", repr(lib)).replace("@SIZE@", str(size)) \
        .replace("@FIELD@", repr(field)).replace("@OUTDIR@", repr(outdir)).replace("@BACK@", str(back)) \
        .replace("@SHAPE@", _shape(size, dims)).replace("@DIMS@", str(dims)).replace("@RATE@", str(rate)) \
        .replace("@DTYPE@", repr(dtype))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    if r.returncode:
        print(r.stderr[-3000:])
        raise SystemExit(r.returncode)
    for name in ("encode", "decode"):
        analyse(os.path.join(outdir, f"stamps_{name}_{field}_{size}.npy"), name)


def analyse(path, name):
    import numpy as np
    a = np.load(path).astype(np.int64)
    hw, t, rt = a[:, 0], a[:, 1:8], a[:, 8:10]
    rel = t - t[:, :1]  # s_memtime bases differ between CUs: per-wave deltas only
    r0 = rt[:, 0].min()
    rs, re = (rt[:, 0] - r0) * 10, (rt[:, 1] - r0) * 10  # ns (100 MHz)
    print(f"== {name}: {len(a)} waves, span {re.max()} ns;  wave start ns p10/50/90/max "
          f"{int(np.percentile(rs, 10))} {int(np.median(rs))} {int(np.percentile(rs, 90))} {rs.max()};"
          f"  end ns p10/50/90/max {int(np.percentile(re, 10))} {int(np.median(re))} {int(np.percentile(re, 90))} {re.max()}")
    labels = (["start", "emax(load)", "transform", "transpose", "planes", "-", "end"] if name == "encode"
              else ["start", "planes", "transpose", "inv-xform", "fast pairs", "copy-in", "end"])
    order = [0, 1, 2, 3, 4, 6] if name == "encode" else [0, 5, 4, 1, 2, 3, 6]
    prev = None
    for k in order:
        col = rel[:, k]
        line = f"  {labels[k]:11s}"
        if prev is not None:
            d = rel[:, k] - rel[:, prev]
            line += f"   phase: mean {int(d.mean()):6d} p50 {int(np.median(d)):6d} max {d.max():6d}"
        print(line)
        prev = k
    simd = ((hw >> 32) << 16) | (((hw >> 13) & 3) << 12) | (((hw >> 12) & 1) << 11) | (((hw >> 8) & 15) << 4) | ((hw >> 4) & 3)
    u, cnt = np.unique(simd, return_counts=True)
    print(f"  distinct SIMDs {len(u)}, waves per SIMD: min {cnt.min()} max {cnt.max()} mean {cnt.mean():.2f}")
    life = rel[:, 6] - rel[:, 0]
    print(f"  wave lifetime: mean {int(life.mean())} p50 {int(np.median(life))} max {life.max()}")


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--field", default="polynomial")
    ap.add_argument("--back", type=int, default=1, help="stamped launches back to back (the last one's stamps)")
    ap.add_argument("--variants", default=",".join(map(str, VARIANTS)), help="build: CUZFP_PROBE values")
    ap.add_argument("--dims", type=int, default=3)
    ap.add_argument("--rate", type=float, default=8.0)
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--lib", default="p9", help="stamps: the build/probe/ subdirectory of the stamped library")
    a = ap.parse_args()
    if a.cmd == "build":
        build(tuple(int(v) for v in a.variants.split(",")))
    elif a.cmd == "stamps":
        od = os.path.join(ROOT, "gpurun_out")
        os.makedirs(od, exist_ok=True)
        stamps(a.size, a.field, od, a.back, a.dims, a.rate, a.dtype, a.lib)
    else:
        run(a.size, a.field, a.dims, a.rate, dtype=a.dtype)
