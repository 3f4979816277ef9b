#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (``--pmc ... --output-format csv``) per kernel.

usage: pmc_summary.py DIR [DIR ...] [--traffic OUT.json] [--launches-per-step N]

Every ``*_counter_collection.csv`` under the given directories is read; counters are
averaged per dispatch of each kernel (short name = the function name without namespaces
or arguments).  ``--traffic`` writes the per-launch HBM bytes that ``bench.py`` puts in
``roofline.traffic``: FETCH_SIZE and WRITE_SIZE are reported in KiB; on gfx950 FETCH_SIZE
counts wide coalesced reads at half their bytes (MI355X_MICROARCH.md, "HBM [CDNA4]"), so
hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  The correction is calibrated for
16-B-per-lane streaming reads; other widths are uncalibrated (the raw values are kept).
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--traffic", default=None)
    ap.add_argument("--workload", default="1m_1080p", help="bench.py --config the passes ran")
    args = ap.parse_args()
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
               "workload": args.workload,
               "correction": "hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halving)",
               "kernels": {}}
        for k in kernels:
            t = table[k]
            rec = {}
            if "FETCH_SIZE" in t and "WRITE_SIZE" in t:
                rec.update(fetch_size_kib=round(t["FETCH_SIZE"], 3), write_size_kib=round(t["WRITE_SIZE"], 3),
                           hbm_bytes_per_launch=int((2 * t["FETCH_SIZE"] + t["WRITE_SIZE"]) * 1024))
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
