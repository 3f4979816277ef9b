#!/usr/bin/env python3
"""Per-dispatch timeline of one bench iteration from a rocprofv3 --kernel-trace CSV:
kernel durations and the idle gaps between them (host launch / sync latency).
usage: trace_gaps.py TRACE_CSV [iteration]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    it = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    seq = []
    for r in rows:
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("gsr::", "").replace("void ", "")
        seq.append((n, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    seq.sort(key=lambda x: x[1])
    starts = [i for i, (n, _, _) in enumerate(seq) if n == "preprocess_kernel"]
    a, b = starts[it], starts[it + 1]
    t0 = seq[a][1]
    busy = gaps = 0.0
    prev_end = None
    for n, s, e in seq[a:b]:
        gap = 0.0 if prev_end is None else (s - prev_end) / 1e3
        busy += (e - s) / 1e3
        gaps += max(gap, 0.0)
        print(f"{n:34s} t={(s - t0) / 1e3:8.1f}us dur={(e - s) / 1e3:7.1f}us gap_before={gap:6.1f}us")
        prev_end = e
    total = (seq[b][1] - t0) / 1e3
    print(f"iteration {total:.1f} us: kernels {busy:.1f} us, gaps {gaps:.1f} us")


if __name__ == "__main__":
    main()
