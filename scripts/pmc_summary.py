#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (``--pmc ... --output-format csv``) per kernel.

usage: pmc_summary.py DIR [DIR ...] [--traffic OUT.json] [--launches-per-step N]

Every ``*_counter_collection.csv`` under the given directories is read; counters are
averaged per dispatch of each kernel (short name = the function name without namespaces
or arguments).  ``--traffic`` writes the per-launch HBM bytes that ``bench.py`` puts in
``roofline.traffic``: FETCH_SIZE and WRITE_SIZE are reported in KiB.  FETCH_SIZE = TCC_EA0_RDREQ
x 64 B (MI355X_MICROARCH.md "HBM [CDNA4]"), so the correction depends on the request size of
the kernel's dominant read pattern.  scripts/ubench/fetch_calib.hip measures each pattern on a
known byte count from a 2 GiB buffer (``--calib DIR``: its FETCH/WRITE passes):
  * stream (coalesced 16-B/lane, F1 / B2 / gather / scan / radix key streams): counted = 1/2 of
    the bytes (128-B requests tallied at 64 B) -> factor 2.0 (calibrated 1.9999).
  * gather (one random 16-B or 48-B record per lane: F6 / B1 / per-tile depth sort): counted =
    64 B per random 16-B access (calibrated: 4.0 counted bytes per useful byte) and 80.6 B per
    random 48-B record (1.68 per useful byte) -- one tallied request per L2 miss.  The request
    size behind a miss is not observable here (64-B request: the count is exact; 128-B line
    fill: x2), so gather kernels use factor 1.0 (``hbm_bytes``, request-exact lower bound) and
    report the x2 bound as ``hbm_bytes_upper``.
hbm_bytes = (factor * FETCH_SIZE + WRITE_SIZE) * 1024.  The raw values are kept as well, and
the library's source stamp (``--lib-stamp``) is recorded so bench.py can drop figures that are
not of the library it loads.
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    head, _, targs = n.partition("<")
    return head.split("::")[-1] + (("<" + targs) if targs else "")


def load(dirs):
    # (kernel, counter) -> list of values (one per dispatch)
    vals = defaultdict(list)
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as fh:
                for row in csv.DictReader(fh):
                    vals[(short(row["Kernel_Name"]), row["Counter_Name"])].append(float(row["Counter_Value"]))
    return vals


# Dominant read pattern per kernel: "stream" (coalesced 16-B/lane: FETCH counts half the bytes)
# or "gather" (random 16/48-B records per lane: one 64-B tally per request).
GATHER_KERNELS = ("blend_forward_kernel", "blend_backward_kernel", "tile_depth_radix", "tile_depth_sort")


def fetch_pattern(kernel: str) -> str:
    return "gather" if kernel.startswith(GATHER_KERNELS) else "stream"


def fetch_factor(kernel: str, calib: dict) -> float:
    return 1.0 if fetch_pattern(kernel) == "gather" else calib.get("stream16", 2.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--traffic", default=None)
    ap.add_argument("--workload", default="1m_1080p", help="bench.py --config the passes ran")
    ap.add_argument("--calib", nargs="*", default=[], help="FETCH/WRITE pass dirs of fetch_calib")
    ap.add_argument("--lib-stamp", default=None, help="source stamp of the profiled libgsr_hip.so")
    args = ap.parse_args()
    calib = {}
    if args.calib:
        cv = load(args.calib)
        moved = 512 * 2 ** 20
        for (k, c), v in cv.items():
            if c == "FETCH_SIZE" and not k.startswith("write"):
                calib[k] = moved / (v[0] * 1024.0)  # bytes moved per reported byte
            if c == "WRITE_SIZE" and k.startswith("write"):
                calib[k] = moved / (v[0] * 1024.0)
        print("calibration (bytes moved / counted bytes):", json.dumps({k: round(v, 4) for k, v in calib.items()}))
    vals = load(args.dirs)
    kernels = sorted({k for k, _ in vals})
    counters = sorted({c for _, c in vals})
    table = {}
    for k in kernels:
        table[k] = {c: sum(v) / len(v) for (kk, c), v in vals.items() if kk == k}
        table[k]["_dispatches"] = max(len(v) for (kk, c), v in vals.items() if kk == k)
    width = max(len(k) for k in kernels) if kernels else 10
    print("kernel".ljust(width), " ".join(c[:18].rjust(18) for c in counters))
    for k in kernels:
        print(k.ljust(width), " ".join(
            (f"{table[k][c]:18.4g}" if c in table[k] else " " * 18) for c in counters))
    if args.traffic:
        out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU, separate passes",
               "workload": args.workload, "lib_stamp": args.lib_stamp,
               "correction": "hbm_bytes = (factor * FETCH_SIZE + WRITE_SIZE) * 1024; stream kernels: factor = "
                             "fetch_calib stream16 (~2.0, 128-B requests tallied at 64 B); gather kernels (random "
                             "16/48-B records): factor 1.0 = one 64-B tally per request (lower bound), "
                             "hbm_bytes_upper at x2 (128-B line fills)",
               "calibration": {k: round(v, 4) for k, v in calib.items()},
               "kernels": {}}
        for k in kernels:
            t = table[k]
            rec = {}
            if "FETCH_SIZE" in t and "WRITE_SIZE" in t:
                f = fetch_factor(k, calib)
                rec.update(fetch_size_kib=round(t["FETCH_SIZE"], 3), write_size_kib=round(t["WRITE_SIZE"], 3),
                           fetch_pattern=fetch_pattern(k), fetch_factor=round(f, 4),
                           hbm_bytes_per_launch=int((f * t["FETCH_SIZE"] + t["WRITE_SIZE"]) * 1024))
                if fetch_pattern(k) == "gather":
                    rec["hbm_bytes_upper_per_launch"] = int((2.0 * t["FETCH_SIZE"] + t["WRITE_SIZE"]) * 1024)
            if "SQ_INSTS_VALU" in t:  # wave-level VALU instructions per launch (issue-bound kernels)
                rec["valu_insts_per_launch"] = int(t["SQ_INSTS_VALU"])
            if "SQ_INSTS_VALU_TRANS_F32" in t:
                rec["valu_trans_insts_per_launch"] = int(t["SQ_INSTS_VALU_TRANS_F32"])
            if rec:
                out["kernels"][k] = rec
        with open(args.traffic, "w") as fh:
            json.dump(out, fh, indent=1)
        print("wrote", args.traffic)


if __name__ == "__main__":
    main()
