#!/usr/bin/env python3
"""Print the top kernels (calls, total ms, average us, %) of a rocprofv3 run_results.db.
usage: scripts/db_top.py DB [N]"""
import sqlite3
import sys

db = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 15
c = sqlite3.connect(db)
for name, calls, total, avg, pct in c.execute("select * from top_kernels limit ?", (n,)):
    # the top_kernels view reports microseconds
    short = name.replace("gsr::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    print(f"{short[:60]:60s} {calls:6d} {total / 1e3:9.1f} ms {avg:8.1f} us {pct:5.1f}%")
