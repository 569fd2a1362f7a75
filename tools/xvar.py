"""Fast timing variants of the 3D float32 kernels (design tool, not the product).

  python tools/xvar.py build NAME "-DFLAG=1 ..." [NAME "FLAGS" ...]   # here
    ("@f64": the double kernels; "@src=DIR": the kernels of another csrc tree,
     e.g. an older commit's, `git archive REV cuzfp_amd/csrc | tar -x -C build/ab`)
  python tools/xvar.py isa NAME [NAME ...]                            # here: ISA histograms
  python tools/xvar.py run [--size S] [--field F] [--dims D --rate R] NAME [NAME ...]   # GPU box
    (variants built with -DCUZFP_XVAR_DIMS=D for 1D / 2D)

Unlike tools/variants.py (a full library per variant), a variant here compiles
only the 3D fast-gather float kernels (-DCUZFP_XVAR); the other scalar
types are stubs built once.  `run` times encode / decode / the step with
hipGraphs and checks the stream and the decoded array against the reference's
SHA-256 digests in tests/golden/golden.json (256^3 rate 8, polynomial and
splitmix fields), so a variant that changes the bits says so.
"""
from __future__ import annotations

import json
import os
import re
import subprocess
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "build", "xvar")
STUB = os.path.join(OUT, "_stub")
LLVM = "/opt/rocm/lib/llvm/bin"


def _stub_objs(unit):
    """Stub objects for every scalar type but `unit`'s, plus the C-ABI."""
    from cuzfp_amd import build as b
    os.makedirs(STUB, exist_ok=True)
    hdrs = [os.path.join(b.CSRC, h) for h in b.HEADERS] + [os.path.join(b.INC, "cuzfp_hip.h")]
    objs, procs = [], []
    for u, flags in (("inst_f32", ["-DCUZFP_XVAR", "-DCUZFP_XVAR_STUB"]), ("inst_f64", ["-DCUZFP_XVAR", "-DCUZFP_XVAR_STUB"]),
                     ("inst_i32", ["-DCUZFP_XVAR", "-DCUZFP_XVAR_STUB"]), ("inst_i64", ["-DCUZFP_XVAR", "-DCUZFP_XVAR_STUB"]), ("capi", [])):
        if u == unit:
            continue
        o = os.path.join(STUB, u + ".o")
        objs.append(o)
        src = os.path.join(b.CSRC, u + ".hip")
        if b._newer(o, [src] + hdrs):
            procs.append(subprocess.Popen([b.HIPCC, *b.CXXFLAGS, *flags, "-c", src, "-o", o]))
    assert all(p.wait() == 0 for p in procs)
    return objs


def _unit(flags: str) -> str:  # "@f64" in a variant's flags: the double kernels
    return "inst_f64" if "@f64" in flags.split() else "inst_f32"


def _src(flags: str) -> str:  # "@src=DIR" in a variant's flags: kernels from another csrc tree (A/B)
    from cuzfp_amd import build as b
    for f in flags.split():
        if f.startswith("@src="):
            return os.path.join(ROOT, f[5:])
    return b.CSRC


def build(pairs):
    from cuzfp_amd import build as b
    procs = []
    for name, flags in pairs:
        d = os.path.join(OUT, name)
        os.makedirs(d, exist_ok=True)
        u = _unit(flags)
        fl = [f for f in flags.split() if not f.startswith("@")]
        procs.append(subprocess.Popen([b.HIPCC, *b.CXXFLAGS, "-DCUZFP_XVAR", *fl, "-c",
                                       os.path.join(_src(flags), u + ".hip"), "-o", os.path.join(d, "inst_f32.o")]))
    assert all(p.wait() == 0 for p in procs)
    for name, flags in pairs:
        d = os.path.join(OUT, name)
        subprocess.check_call([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o",
                               os.path.join(d, "libcuzfp_hip.so"), os.path.join(d, "inst_f32.o"),
                               *_stub_objs(_unit(flags))])
        with open(os.path.join(d, "flags.txt"), "w") as f:
            f.write(flags + "\n")
    print("built", [n for n, _ in pairs])


# Issue classes measured on gfx950 (profiles/r02_opcost.txt): "fast" VOP2/VOP1
# ops issue every 2 cycles with >= 2 waves per SIMD, "slow" ones every ~3-4.
FAST = re.compile(r"^v_(add_u32|sub_u32|subrev_u32|ashrrev_i32|lshrrev_b32|lshlrev_b32|xor_b32|and_b32|or_b32|"
                  r"not_b32|mov_b32|mul_f32|lshlrev_b16)_e32$")


def isa(names):
    for name in names:
        d = os.path.join(OUT, name)
        o = os.path.join(d, "inst_f32.o")
        co, fat = os.path.join(d, "f32.co"), os.path.join(d, "fat.bin")
        subprocess.check_call(["objcopy", f"--dump-section=.hip_fatbin={fat}", o])
        subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}", f"--output={co}"])
        dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co],
                             capture_output=True, text=True, check=True).stdout
        with open(os.path.join(d, "f32.dis"), "w") as f:
            f.write(dis)
        kern, hist = None, {}
        for line in dis.splitlines():
            m = re.match(r"^[0-9a-f]+ <(_Z.*)>:$", line)
            if m:
                kern = m.group(1)
                hist[kern] = Counter()
                continue
            if kern and line.startswith("\t"):
                hist[kern][line.split()[0]] += 1
        for k, h in hist.items():
            valu = sum(v for i, v in h.items() if i.startswith("v_"))
            fast = sum(v for i, v in h.items() if FAST.match(i))
            salu = sum(v for i, v in h.items() if i.startswith("s_") and not i.startswith("s_waitcnt"))
            lds = sum(v for i, v in h.items() if i.startswith("ds_"))
            print(f"{name:10s} {k[:60]:60s} VALU {valu:6d} (fast {fast:5d}, slow {valu - fast:5d}) "
                  f"SALU {salu:5d} LDS {lds:4d} waitcnt {h['s_waitcnt']:4d}")


CODE = """
import os, sys, json, hashlib, torch
sys.path.insert(0, {root!r})
os.environ['CUZFP_HIP_LIB'] = {lib!r}
import numpy as np
import cuzfp_amd as cz
from cuzfp_amd.datagen import polynomial_field, splitmix_uniform
shape = ({size},)*{dims}
arr = polynomial_field(shape, {dtype!r}) if {field!r} == 'polynomial' else splitmix_uniform(shape, {dtype!r})
x = torch.from_numpy(arr).cuda()
mb = cz.rate_to_maxbits({rate}, arr.dtype, {dims})
w = cz.encode(x, mb); y = cz.decode(w, shape, x.dtype, mb)
torch.cuda.synchronize()
gold = json.load(open(os.path.join({root!r}, 'tests', 'golden', 'golden.json')))['cases']
key = 'baseline/%dd_%s_%s_r%d/%s' % ({dims}, 'f32' if {dtype!r} == 'float32' else 'f64', '1M' if {size} == 1 << 20 else str({size}), {rate}, {field!r})
ok = None
if key in gold:
    s = hashlib.sha256(w.cpu().numpy().tobytes()).hexdigest() == gold[key]['stream_sha256']
    t = hashlib.sha256(y.cpu().numpy().tobytes()).hexdigest() == gold[key]['decoded_sha256']
    ok = 'ok' if s and t else 'STREAM DIFFERS' if not s else 'DECODE DIFFERS'
def t(fn):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(20): fn()
    g.replay(); torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    r = []
    for _ in range(11):
        torch.cuda.synchronize(); e0.record()
        g.replay(); g.replay()
        e1.record(); torch.cuda.synchronize()
        r.append(e0.elapsed_time(e1) / 40 * 1000)
    return round(sorted(r)[5], 2)
def step():
    cz.encode(x, mb, out=w); cz.decode(w, shape, x.dtype, mb, out=y)
print(json.dumps(dict(enc_us=t(lambda: cz.encode(x, mb, out=w)), dec_us=t(lambda: cz.decode(w, shape, x.dtype, mb, out=y)),
                      step_us=t(step), parity=ok)))
"""


def run(names, size, fields, dims=3, rate=8, dtype="float32"):
    for field in fields:
        for name in names:
            lib = os.path.join(OUT, name, "libcuzfp_hip.so")
            code = CODE.format(root=ROOT, lib=lib, size=size, field=field, dims=dims, rate=rate, dtype=dtype)
            r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
            if r.returncode:
                print(name, "FAILED", r.stderr[-800:], flush=True)
                sys.exit(r.returncode)
            print(f"{name:12s} {field:10s} {dims}D {size} r{rate} {r.stdout.strip()}", flush=True)


if __name__ == "__main__":
    cmd = sys.argv[1]
    if cmd == "build":
        a = sys.argv[2:]
        build(list(zip(a[0::2], a[1::2])))
    elif cmd == "isa":
        isa(sys.argv[2:])
    elif cmd == "run":
        a = sys.argv[2:]
        size, fields, dims, rate, dtype = 256, ["polynomial"], 3, 8, "float32"
        while a and a[0].startswith("--"):
            if a[0] == "--size":
                size = int(a[1])
            elif a[0] == "--field":
                fields = a[1].split(",")
            elif a[0] == "--dims":
                dims = int(a[1])
            elif a[0] == "--rate":
                rate = int(a[1])
            elif a[0] == "--dtype":
                dtype = a[1]
            a = a[2:]
        run(a, size, fields, dims, rate, dtype)
