#!/usr/bin/env python3
"""Print the top kernels of a rocprofv3 --stats summary: tools/top_kernels.py <kernel_stats.csv> [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 15
for r in rows[:n]:
    name = r["Name"]
    name = name.replace("void ", "").replace("plssvm_mi::(anonymous namespace)::", "").split("(")[0]
    print(f"{name[:60]:60s} calls {int(r['Calls']):6d}  avg {float(r['AverageNs']) / 1e3:10.1f} us  {float(r['Percentage']):6.2f} %")
