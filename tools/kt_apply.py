#!/usr/bin/env python3
"""Median duration of each pipeline launch kind in a kernel trace (grid size = role set)."""
import collections
import csv
import statistics
import sys

for d in sys.argv[1:]:
    rows = [r for r in csv.DictReader(open(f"{d}/kt_kernel_trace.csv")) if "pipeline" in r["Kernel_Name"]]
    by = collections.defaultdict(list)
    for r in rows:
        by[int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    print(d, {g: (len(v), round(statistics.median(v), 1)) for g, v in sorted(by.items(), key=lambda x: -len(x[1]))[:3]})
