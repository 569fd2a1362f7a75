"""HBM traffic per codec launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs.

    python tools/traffic.py gpurun_out/pmc_<tag> [--workload 3d_float32_256^3_rate8] [--out profiles/traffic_latest.json]

Corrections (MI355X_MICROARCH.md, section HBM): FETCH_SIZE / WRITE_SIZE are in
KiB, counted at the L2's memory side; on gfx950 FETCH_SIZE reports exactly half
the bytes of a wide coalesced streaming read (16 B per lane, which is what both
kernels issue: the encoder's block-row gathers and the decoder's stream
copy-in), so it is doubled; WRITE_SIZE is exact for 16-B-per-lane stores (the
encoder's stream copy-out, the decoder's row scatters).  The median over all
dispatches of each kernel is reported.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics


def collect(root: str, counter: str) -> dict[str, list[float]]:
    out: dict[str, list[float]] = {}
    for f in sorted(glob.glob(os.path.join(root, "**", "run_counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter or "cuzfp::zfp_" not in r["Kernel_Name"]:
                continue
            kind = "encode" if "zfp_encode" in r["Kernel_Name"] else "decode"
            out.setdefault(kind, []).append(float(r["Counter_Value"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--workload", default="3d_float32_256^3_rate8")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    fetch = collect(a.root, "FETCH_SIZE")
    write = collect(a.root, "WRITE_SIZE")
    res = {"workload": a.workload, "source": os.path.basename(a.root.rstrip("/")),
           "method": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes; KiB x 1024; "
                     "FETCH_SIZE x 2 (gfx950 16-B/lane streaming-read correction)"}
    for kind in ("encode", "decode"):
        if kind in fetch and kind in write:
            fb = 2 * statistics.median(fetch[kind]) * 1024
            wb = statistics.median(write[kind]) * 1024
            res[f"{kind}_fetch_bytes_per_launch"] = int(fb)
            res[f"{kind}_write_bytes_per_launch"] = int(wb)
            res[f"{kind}_hbm_bytes_per_launch"] = int(fb + wb)
            res[f"{kind}_dispatches"] = len(fetch[kind])
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)
            fh.write("\n")


if __name__ == "__main__":
    main()
