#!/usr/bin/env python3
"""Average counters per dispatch, grouped by grid size (tools/pmc_apply.sh / pmc_ingest.sh output
dirs); KSUB selects the kernel (default: the pipeline kernel)."""
import collections
import csv
import os
import sys

KSUB = os.environ.get("KSUB", "pipeline")

for d in sys.argv[1:]:
    rows = list(csv.DictReader(open(f"{d}/pm_counter_collection.csv")))
    per = collections.defaultdict(dict)
    for r in rows:
        if KSUB not in r["Kernel_Name"]:
            continue
        per[(r["Dispatch_Id"], r["Grid_Size"])][r["Counter_Name"]] = float(r["Counter_Value"])
    by = collections.defaultdict(list)
    for (_, g), v in per.items():
        by[g].append(v)
    for g, vs in sorted(by.items(), key=lambda x: -len(x[1]))[:2]:
        keys = sorted(vs[0])
        print(d, "grid", g, "n", len(vs), {k: round(sum(v.get(k, 0) for v in vs) / len(vs)) for k in keys})
