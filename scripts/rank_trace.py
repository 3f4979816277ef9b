#!/usr/bin/env python3
"""Per-kernel durations of the replayed (one rank at a time) steps of a band_sim.py --cpp run,
from its rocprofv3 kernel trace: the live steps (every rank in its own host thread, concurrent on
the GPU) are dropped by keeping only the dispatches the main thread made after the first worker
thread's; those are the ranks' eager / captured / replayed steps run alone.  Prints per kernel: calls, median / mean us, and the
median step's share.  usage: rank_trace.py trace_kernel_trace.csv [--world 8]"""
import argparse
import csv
import re
import statistics


def short(name: str) -> str:
    n = name.replace("void ", "").replace("gsr::(anonymous namespace)::", "").replace("at::native::", "")
    m = re.match(r"([\w:]+(?:<[^()]*?>)?)", n)
    return m.group(1) if m else n[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    args = ap.parse_args()
    recs = sorted(csv.DictReader(open(args.trace)), key=lambda r: int(r["Start_Timestamp"]))
    main_tid = recs[-1]["Thread_Id"]  # the replays come last, from the main thread
    last_worker = max(int(r["End_Timestamp"]) for r in recs if r["Thread_Id"] != main_tid)
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in recs]
    alone = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in recs
             if r["Thread_Id"] == main_tid and int(r["Start_Timestamp"]) > last_worker]
    by = {}
    for s, e, n in alone:
        by.setdefault(n, []).append((e - s) / 1e3)
    tot = sum(sum(v) for v in by.values())
    print(f"dispatches {len(rows)}, the main thread's after the live steps {len(alone)}")
    for n, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        print(f"{n[:58]:58s} calls {len(v):5d} median_us {statistics.median(v):8.1f} mean_us {statistics.mean(v):8.1f}"
              f"  {sum(v) / tot * 100:5.1f}%")


if __name__ == "__main__":
    main()
