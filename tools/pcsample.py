"""Summarise rocprofv3 stochastic PC-sampling output (design tool, not the product).

    python tools/pcsample.py DIR [--kernel REGEX] [--top N]

Reads every *pc_sampling*.csv under DIR (rocprofv3 --pc-sampling-beta-enabled
--pc-sampling-method stochastic --output-format csv) and prints, per kernel:
  - the share of samples by stall reason (and issued vs not issued),
  - the top N instructions by sample count with their stall-reason split,
  - the samples by code section (contiguous PC ranges split at branch targets
    are too fine; sections are taken from the instruction text's position in
    the kernel: the caller maps PC offsets to phases with --sections).
Column names are matched loosely (rocprofv3's CSV header varies by version).
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import gzip
import os
import re
import sys


def _open(path):
    return gzip.open(path, "rt") if path.endswith(".gz") else open(path, newline="")


def _col(header, *keys):
    for k in keys:
        for h in header:
            if h.lower() == k.lower():
                return h
    for k in keys:
        for h in header:
            if k.lower() in h.lower():
                return h
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default=".")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--sections", default="", help="comma list of name:pc_start (hex offsets) to bucket samples")
    a = ap.parse_args()
    files = sorted(glob.glob(os.path.join(a.dir, "**", "*pc_sampling*.csv*"), recursive=True))
    if not files:
        print("no pc sampling csv under", a.dir)
        return 1
    kre = re.compile(a.kernel)
    # dispatch id -> kernel name, from the kernel trace if present
    names = {}
    for kt in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        with _open(kt) as fh:
            r = csv.DictReader(fh)
            dc = _col(r.fieldnames, "Dispatch_Id")
            kc = _col(r.fieldnames, "Kernel_Name")
            for row in r:
                names[row[dc]] = row[kc]
    secs = []
    for s in filter(None, a.sections.split(",")):
        n, p = s.split(":")
        secs.append((int(p, 16), n))
    secs.sort()
    for f in files:
        with _open(f) as fh:
            r = csv.DictReader(fh)
            hdr = r.fieldnames
            print("file", f)
            print("columns", hdr)
            c_inst = _col(hdr, "Instruction")
            c_stall = _col(hdr, "Stall_Reason", "Stall")
            c_iss = _col(hdr, "Wave_Issued", "Issued")
            c_disp = _col(hdr, "Dispatch_Id")
            c_kern = _col(hdr, "Kernel_Name")
            c_pc = _col(hdr, "Code_Object_Offset", "Pc", "PC")
            c_type = _col(hdr, "Inst_Type", "Instruction_Type")
            per_k = collections.defaultdict(lambda: {"n": 0, "stall": collections.Counter(), "inst": collections.Counter(),
                                                     "inst_stall": collections.defaultdict(collections.Counter),
                                                     "issued": collections.Counter(), "type": collections.Counter(),
                                                     "sec": collections.Counter(), "pc": {}})
            for row in r:
                k = row.get(c_kern) if c_kern else names.get(row.get(c_disp, ""), row.get(c_disp, "?"))
                k = k or "?"
                if not kre.search(k):
                    continue
                d = per_k[k]
                d["n"] += 1
                st = row.get(c_stall, "?") if c_stall else "?"
                iss = row.get(c_iss, "?") if c_iss else "?"
                ins = row.get(c_inst, "?") if c_inst else "?"
                pc = row.get(c_pc, "") if c_pc else ""
                d["stall"][st] += 1
                d["issued"][iss] += 1
                if c_type:
                    d["type"][row.get(c_type, "?")] += 1
                key = (pc, ins)
                d["inst"][key] += 1
                d["inst_stall"][key][st] += 1
                if secs and pc:
                    try:
                        v = int(pc, 16) if pc.startswith("0x") else int(pc)
                    except ValueError:
                        v = -1
                    name = "?"
                    for p0, n in secs:
                        if v >= p0:
                            name = n
                    d["sec"][name] += 1
        for k, d in per_k.items():
            n = d["n"]
            print()
            print("=" * 100)
            print(f"kernel {k}: {n} samples")
            print("  issued:", ", ".join(f"{x}={c} ({100.0 * c / n:.1f}%)" for x, c in d["issued"].most_common()))
            print("  stall reasons:")
            for x, c in d["stall"].most_common():
                print(f"    {x:40s} {c:8d}  {100.0 * c / n:5.1f}%")
            if d["type"]:
                print("  instruction types:")
                for x, c in d["type"].most_common():
                    print(f"    {x:40s} {c:8d}  {100.0 * c / n:5.1f}%")
            if d["sec"]:
                print("  sections:")
                for x, c in d["sec"].most_common():
                    print(f"    {x:40s} {c:8d}  {100.0 * c / n:5.1f}%")
            print(f"  top {a.top} instructions:")
            for (pc, ins), c in d["inst"].most_common(a.top):
                split = ", ".join(f"{s}:{v}" for s, v in d["inst_stall"][(pc, ins)].most_common(3))
                print(f"    {c:7d} {100.0 * c / n:5.2f}%  {pc:>8s}  {ins[:60]:60s}  {split}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
