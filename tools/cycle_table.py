"""Issue-cycle table of the 3D float32 kernels: where a block's cycles go (design tool).

    python tools/cycle_table.py [--obj build/obj/inst_f32.o] [--ctr profiles/r06_counters.txt]
                                [--enc-us E --dec-us D]

For each of the headline kernels (zfp_encode / zfp_decode<float, 3, FAST, PRIO>)
the main path's ISA is cut into sections -- encoder: prologue (gathers,
exponent, quantisation, lifting, negabinary), transpose, one plane step;
decoder: prologue (copy-in, header), one plane step, finish (transpose,
inverse lifting, dequantisation, stores) -- and each section's VALU
instructions are priced at the issue cost measured on gfx950 with four waves
a SIMD (profiles/r02_opcost.txt: fast VOP1/VOP2 add/sub/logic/constant-shift
/move 2.03 cycles, every other VALU 3.19).  Plane steps are scaled by the
dynamic step counts of the polynomial field (tools/dec_paths.cpp,
tools/coder_stats.cpp: 29.5 steps a wave).  A SIMD runs four waves of 64
blocks, so SIMD cycles per block = a wave's issue cycles / 64.  Against it:
the kernel's measured time in SIMD cycles per block (2.4 GHz, 256 blocks a
SIMD at 256^3) and the budget the north star's 70 % of HBM peak leaves
(83.9 MB a launch / 5.6 TB/s = 14.98 us = 140 cycles a block).
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
from statistics import median

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
FAST = re.compile(r"^v_(add_u32|sub_u32|subrev_u32|ashrrev_i32|lshrrev_b32|lshlrev_b32|xor_b32|and_b32|or_b32|"
                  r"not_b32|mov_b32|mul_f32|lshlrev_b16)_e32$")
C_FAST, C_SLOW = 2.03, 3.19     # cycles a wave-instruction, four waves a SIMD (r02_opcost.txt)
CLOCK_GHZ = 2.4                 # MI355X peak engine clock (MI355X_MICROARCH.md)
BLOCKS_PER_SIMD = 256           # 256^3 f32: 262,144 blocks on 1,024 SIMDs
BUDGET_US = 83886080 / (0.7 * 8.0e12) * 1e6   # 70 % of HBM peak for one launch's algorithmic bytes
STEPS = 29.47                   # plane steps a wave, polynomial field (dec_paths: 29.47; encoder the same walk)
DEC_RARE, ENC_WIDE = 2.50, 2.6  # wave-steps a wave on the decoder's rare path / the encoder's wide step


def disassemble(obj: str) -> str:
    work = os.path.join(ROOT, "build", "isa")
    os.makedirs(work, exist_ok=True)
    fat, co = os.path.join(work, "ct_fat.bin"), os.path.join(work, "ct_f32.co")
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
            out[name].append(line.split("//")[0].strip())
    return out


def mix(lines) -> tuple:
    ops = [l.split()[0] for l in lines if l]
    valu = [o for o in ops if o.startswith("v_")]
    fast = sum(1 for o in valu if FAST.match(o))
    return len(valu), fast, len(valu) - fast


def cyc(fast: float, slow: float) -> float:
    return fast * C_FAST + slow * C_SLOW


def first(lines, pred, start=0):
    for i in range(start, len(lines)):
        if pred(lines[i]):
            return i
    return len(lines)


def sgpr_perm(l: str) -> bool:  # a transpose's v_perm_b32 (selector in an SGPR or a literal)
    return l.startswith("v_perm_b32") and not re.search(r",\s*v\d+\s*$", l)


def steps_between(lines, a, b, start_pred):
    """the instruction ranges between consecutive lines matching start_pred in [a, b)"""
    idx = [i for i in range(a, b) if start_pred(lines[i])]
    return [lines[i:j] for i, j in zip(idx, idx[1:])]


def row(name, n, f, s, count=1.0):
    c = cyc(f, s) * count
    return (name, n * count, f * count, s * count, c, c / 64.0)


def table(ks):
    rows = {}
    for name, lines in ks.items():
        enc = re.search(r"zfp_encodeIfLi3ELb1ELb1ELb1E", name)  # FAST, ALIGNED, PRIO
        dec = re.search(r"zfp_decodeIfLi3ELb1ELb1E", name)      # FAST, PRIO
        if not (enc or dec):
            continue
        if enc:
            t0 = first(lines, sgpr_perm)
            t1 = first(lines, lambda l: l.startswith("ds_read_b32"), t0)
            # a plane step: from one pair of ds_or_b64 (the put) to the next
            e = first(lines, lambda l: l.startswith("s_endpgm"), t1)  # in-line steps only (wide steps are laid out after it)
            puts = [i for i in range(t1, e) if lines[i].startswith("ds_or_b64") and
                    i + 1 < len(lines) and lines[i + 1].startswith("ds_or_b64")]
            steps = [lines[i + 2:j + 2] for i, j in zip(puts, puts[1:]) if j - i < 80]
            st = sorted(steps, key=len)[len(steps) // 2] if steps else []
            r = [row("prologue: gathers, exponent, quantisation, lifting, negabinary", *mix(lines[:t0])),
                 row("bit-plane transpose (64 x 32 bits)", *mix(lines[t0:t1])),
                 row(f"plane steps ({STEPS} a wave, one-put step)", *mix(st), count=STEPS)]
            rows["encode"] = r
        else:
            p0 = first(lines, lambda l: l.startswith("ds_read2st64"))
            t0 = first(lines, sgpr_perm, p0)
            steps = steps_between(lines, p0, t0, lambda l: l.startswith("ds_read2st64_b32") and "offset1:1" in l
                                  and "offset:" not in l)
            # each step issues two ds_read2st64 (group window, verbatim window): pair them
            whole = [a + b for a, b in zip(steps[0::2], steps[1::2])]
            st = sorted(whole, key=len)[len(whole) // 2] if whole else []
            e = first(lines, lambda l: l.startswith("s_endpgm"), t0)
            r = [row("prologue: copy-in, tables, header", *mix(lines[:p0])),
                 row(f"plane steps ({STEPS} a wave, common path)", *mix(st), count=STEPS),
                 row("finish: transpose, inverse lifting, dequantisation, stores", *mix(lines[t0:e + 1]))]
            rows["decode"] = r
    return rows


def counters(path: str) -> dict:
    """SQ_INSTS_* / SQ_WAVES of the 3D f32 kernels in a tools/counters.py report"""
    out, kind, vals = {}, None, {}
    for line in open(path):
        m = re.match(r"^zfp_(encode|decode)<float, 3, true, true", line)
        if m:
            kind, vals = m.group(1), {}
            continue
        m = re.match(r"^\s+(SQ_\w+)\s+([0-9.e+]+)", line)
        if kind and m:
            vals[m.group(1)] = float(m.group(2))
            if "SQ_WAVES" in vals:
                out[kind] = {k[len("SQ_INSTS_"):]: v / vals["SQ_WAVES"] for k, v in vals.items()
                             if k.startswith("SQ_INSTS_")}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--obj", default=os.path.join(ROOT, "build", "obj", "inst_f32.o"))
    ap.add_argument("--enc-us", type=float, default=None, help="measured encode time (us) for the wall column")
    ap.add_argument("--dec-us", type=float, default=None)
    ap.add_argument("--ctr", default=None, help="tools/counters.py output: dynamic VALU a wave beside the static count")
    a = ap.parse_args()
    rows = table(kernels(disassemble(a.obj)))
    dyn = counters(a.ctr) if a.ctr else {}
    budget = BUDGET_US * 1e-6 * CLOCK_GHZ * 1e9 / BLOCKS_PER_SIMD
    print(f"issue cost: fast {C_FAST} / slow {C_SLOW} cycles a wave-instruction (4 waves a SIMD); "
          f"SIMD cycles a block = wave cycles / 64; clock {CLOCK_GHZ} GHz")
    print(f"70 % of HBM peak: {BUDGET_US:.2f} us a launch = {budget:.0f} SIMD cycles a block\n")
    hdr = f"{'section':66s} {'VALU':>7s} {'fast':>7s} {'slow':>7s} {'cyc/wave':>9s} {'cyc/block':>9s}"
    for kind in ("encode", "decode"):
        if kind not in rows:
            continue
        print(f"== zfp_{kind}<float, 3> (256^3 rate 8)")
        print(hdr)
        tot = [0.0] * 5
        for r in rows[kind]:
            print(f"{r[0]:66s} {r[1]:7.0f} {r[2]:7.0f} {r[3]:7.0f} {r[4]:9.0f} {r[5]:9.1f}")
            for i in range(5):
                tot[i] += r[i + 1]
        extra = (DEC_RARE if kind == "decode" else ENC_WIDE)
        print(f"{'(not priced: ' + ('rare-path steps' if kind == 'decode' else 'wide steps') + f', ~{extra} a wave)':66s}")
        print(f"{'total, priced':66s} {tot[0]:7.0f} {tot[1]:7.0f} {tot[2]:7.0f} {tot[3]:9.0f} {tot[4]:9.1f}")
        if kind in dyn and "VALU" in dyn[kind]:
            d = dyn[kind]
            print(f"{'dynamic (SQ counters): VALU a wave, SQ_INSTS_VALU / SQ_WAVES':66s} {d['VALU']:7.0f}")
            other = ", ".join(f"{k} {d[k]:.0f}" for k in ("SALU", "LDS", "BRANCH", "VMEM", "SMEM") if k in d)
            print(f"{'  beside them a wave issues (not priced): ' + other}")
        us = a.enc_us if kind == "encode" else a.dec_us
        if us:
            wall = us * 1e-6 * CLOCK_GHZ * 1e9 / BLOCKS_PER_SIMD
            print(f"{'measured kernel time ' + f'{us:.1f} us':66s} {'':7s} {'':7s} {'':7s} {'':9s} {wall:9.1f}")
            print(f"{'  VALU-priced share of the wall time':66s} {'':31s} {100 * tot[4] / wall:8.0f}%")
            print(f"{'  to reach 70 % of HBM: cut (cycles a block)':66s} {'':31s} {wall - budget:9.1f}")
        print()


if __name__ == "__main__":
    main()
