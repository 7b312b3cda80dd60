#!/usr/bin/env python3
"""Median duration per kernel (name, grid) over the last N dispatches of a rocprofv3 kernel trace.
usage: tools/trace_summary.py <kernel_trace.csv> [N]"""
import collections
import csv
import statistics as st
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rs = rows[-int(sys.argv[2]) if len(sys.argv) > 2 else 0:]
d = collections.defaultdict(list)
for r in rs:
    d[(r["Kernel_Name"][:70], r["Grid_Size_X"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k[0]:72s} grid={k[1]:>8s} n={len(v):5d} med={st.median(v):8.2f}us sum={sum(v):9.1f}us")
span = (int(rs[-1]["End_Timestamp"]) - int(rs[0]["Start_Timestamp"])) / 1e3
print(f"span {span:.1f} us over {len(rs)} dispatches")
