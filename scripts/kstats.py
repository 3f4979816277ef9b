#!/usr/bin/env python3
"""Per-kernel average durations of rocprofv3 kernel_stats.csv files, side by side.
usage: scripts/kstats.py A_kernel_stats.csv [B_kernel_stats.csv ...]"""
import csv
import sys


def load(path):
    out = {}
    for r in list(csv.reader(open(path)))[1:]:
        name = r[0].replace("gsr::(anonymous namespace)::", "").replace("void ", "")
        name = name.split("(")[0][:46]
        out[name] = (int(r[1]), float(r[3]) / 1000)
    return out


tabs = [load(p) for p in sys.argv[1:]]
names = sorted({k for t in tabs for k in t}, key=lambda k: -max(t.get(k, (0, 0))[1] * t.get(k, (0, 0))[0] for t in tabs))
calls0 = max(v[0] for v in tabs[0].values())
print(f"{'kernel':46s} " + " ".join(f"{'us/call':>9s}" for _ in tabs))
for k in names:
    vals = [t.get(k) for t in tabs]
    if all(v is None or v[0] < 20 for v in vals):
        continue
    print(f"{k:46s} " + " ".join(f"{v[1] * v[0] / (calls0 / 2 if False else 1) / max(v[0], 1):9.1f}x{v[0]:<4d}" if v else f"{'-':>14s}" for v in vals))
