"""Per-kernel, per-phase ISA histogram of the 3D float32 codec kernels (design tool).

  python tools/isa_hist.py [OBJ]      # OBJ: an inst_f32.o (default: build/obj/inst_f32.o)

Disassembles the gfx950 code object of the translation unit and, for the
fast-gather 3D kernels (zfp_encode<float,3,true,true,*>, zfp_decode<float,3,true,*>),
counts instructions by mnemonic and by phase, with each VALU op classed by its
measured issue cost on gfx950 (profiles/r02_opcost.txt, profiles/r03_xvar.txt):
"fast" VOP1/VOP2 add/sub/logic/constant-shift/move ops issue every ~2 (ubench)
to ~2.75 (in the kernel) cycles with several waves a SIMD, every other VALU op
("slow": VOP3, compares, min/max, 64-bit shifts, v_cndmask...) every ~3.2-4.3.

Phases are cut at the first instruction of each: encoder -- prologue (gathers,
exponent, quantisation, lifting: up to the first v_perm_b32), transpose (up to
the first ds_read_b32 of the plane coder's tables), plane coder and copy-out;
decoder -- prologue (copy-in, header), plane decoder (up to the first v_perm_b32
of the inverse transpose), transpose + inverse lifting + stores.  Counts are
static (each instruction once): the plane loops are unrolled, so a phase's
count is close to what one wave executes, except for the rare paths (the
encoder's wide step, the decoder's lut_finish / general decoder), which are
listed separately: the compiler lays them out after the main path's
s_endpgm.  The dynamic per-wave counts are SQ_INSTS_VALU / SQ_WAVES in
profiles/r03_counters.txt.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
FAST = re.compile(r"^v_(add_u32|sub_u32|subrev_u32|ashrrev_i32|lshrrev_b32|lshlrev_b32|xor_b32|and_b32|or_b32|"
                  r"not_b32|mov_b32|mul_f32|lshlrev_b16)_e32$")


def disassemble(obj: str) -> str:
    work = os.path.join(ROOT, "build", "isa")
    os.makedirs(work, exist_ok=True)
    fat, co = os.path.join(work, "fat.bin"), os.path.join(work, "f32.co")
    subprocess.check_call(["objcopy", f"--dump-section=.hip_fatbin={fat}", obj])
    subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}", f"--output={co}"])
    return subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co],
                          capture_output=True, text=True, check=True).stdout


def kernels(dis: str) -> dict:
    out, name = {}, None
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <(_Z.*)>:$", line)
        if m:
            name = m.group(1)
            out[name] = []
        elif name and line.startswith("\t"):
            out[name].append(line.split()[0])
    return out


def summary(ops: list) -> str:
    h = Counter(ops)
    valu = sum(v for k, v in h.items() if k.startswith("v_"))
    fast = sum(v for k, v in h.items() if FAST.match(k))
    salu = sum(v for k, v in h.items() if k.startswith("s_") and k not in ("s_waitcnt", "s_nop"))
    lds = sum(v for k, v in h.items() if k.startswith("ds_"))
    vmem = sum(v for k, v in h.items() if k.startswith(("global_", "buffer_")))
    cyc = 2.75 * fast + 4.3 * (valu - fast)
    top = ", ".join(f"{k} {v}" for k, v in h.most_common(12))
    return (f"VALU {valu:5d} (fast {fast:5d}, slow {valu - fast:5d}; ~{cyc:7.0f} issue cycles at 2.75/4.3)  "
            f"SALU {salu:4d}  LDS {lds:3d}  VMEM {vmem:3d}  s_waitcnt {h['s_waitcnt']:3d}  s_nop {h['s_nop']:3d}\n"
            f"      top: {top}")


def vgpr_counts(co: str) -> dict:
    """kernel name -> .vgpr_count from the code object's metadata notes"""
    notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co],
                           capture_output=True, text=True, check=True).stdout
    out, vg = {}, None
    for line in notes.splitlines():
        m = re.match(r"\s+\.vgpr_count:\s+(\d+)", line)
        if m:
            vg = int(m.group(1))
        m = re.match(r"\s+\.name:\s+(_Z\S+)", line)
        if m:
            out[m.group(1)] = vg
    return out


def first(ops, pred, start=0):
    for i in range(start, len(ops)):
        if pred(ops[i]):
            return i
    return len(ops)


def main():
    obj = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "build", "obj", "inst_f32.o")
    ks = kernels(disassemble(obj))
    meta = vgpr_counts(os.path.join(ROOT, "build", "isa", "f32.co"))
    for name, ops in ks.items():
        enc = re.search(r"zfp_encodeI[fd]Li3ELb1ELb1ELb(\d)", name)
        # zfp_decode<Scalar, 3, FAST=true, PRIO, ...>
        dec = re.search(r"zfp_decodeI[fd]Li3ELb1ELb(\d)E", name)
        if not (enc or dec):
            continue
        kind = "encode" if enc else "decode"
        prio = (enc or dec).group(1) == "1"
        print(f"== zfp_{kind}<float,3,FAST{',ALIGNED' if enc else ''},PRIO={int(prio)}>: {len(ops)} instructions, "
              f"{meta.get(name, '?')} VGPRs")
        print("   whole  " + summary(ops))
        if enc:
            t0 = first(ops, lambda o: o == "v_perm_b32")
            t1 = first(ops, lambda o: o == "ds_read_b32", t0)
            print("   prologue (gathers, exponent, quantisation, lifting)\n          " + summary(ops[:t0]))
            print("   transpose\n          " + summary(ops[t0:t1]))
            e = first(ops, lambda o: o == "s_endpgm", t1)
            print("   plane coder (one-put steps, wide steps) and copy-out\n          " + summary(ops[t1:e + 1]))
            e = first(ops, lambda o: o == "s_endpgm", t1)
            if e + 1 < len(ops):
                print("   out-of-line blocks after s_endpgm\n          " + summary(ops[e + 1:]))
        else:
            p0 = first(ops, lambda o: o.startswith("ds_read2st64"))
            t0 = first(ops, lambda o: o == "v_perm_b32", p0)
            e = first(ops, lambda o: o == "s_endpgm", t0)
            print("   prologue (copy-in, header)\n          " + summary(ops[:p0]))
            print("   plane decoder, fast steps (in line)\n          " + summary(ops[p0:t0]))
            print("   transpose, inverse lifting, dequantisation, stores\n          " + summary(ops[t0:e + 1]))
            print("   out-of-line rare paths after s_endpgm (lut_finish, general decoder)\n          "
                  + summary(ops[e + 1:]))


if __name__ == "__main__":
    main()
