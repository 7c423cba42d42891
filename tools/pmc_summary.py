#!/usr/bin/env python3
"""Per-launch HBM traffic of one kernel from two rocprofv3 --pmc runs (MI355X_MICROARCH.md "HBM").

usage: pmc_summary.py <FETCH_SIZE counter_collection.csv> <WRITE_SIZE counter_collection.csv>
                      <kernel substring> <group> <config> [out.json]

FETCH_SIZE / WRITE_SIZE are KiB per dispatch. On gfx950 FETCH_SIZE tallies the 128-B requests of
16-B-per-lane streaming reads at 64 B, so it is doubled; WRITE_SIZE is exact for 16-B stores.
Only dispatches with the modal grid size are averaged: the steady-state launches that carry every
pipeline stage."""
import csv
import json
import statistics
import sys
from collections import Counter


def per_dispatch(path, counter, flt):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if flt in r["Kernel_Name"] and r["Counter_Name"] == counter:
                rows.append((int(r["Grid_Size"]), float(r["Counter_Value"]) * 1024.0))
    if not rows:
        raise SystemExit(f"{path}: no {counter} rows for {flt}")
    grid = Counter(g for g, _ in rows).most_common(1)[0][0]
    return grid, [v for g, v in rows if g == grid]


def main():
    fpath, wpath, flt, group, config = sys.argv[1:6]
    gf, f = per_dispatch(fpath, "FETCH_SIZE", flt)
    gw, w = per_dispatch(wpath, "WRITE_SIZE", flt)
    fetch, write = 2.0 * statistics.mean(f), statistics.mean(w)
    out = {"kernel": flt, "group": int(group), "config": config, "grid_size": [gf, gw],
           "dispatches": [len(f), len(w)], "fetch_size_raw_bytes": statistics.mean(f),
           "fetch_bytes": fetch, "write_bytes": write, "traffic_bytes_per_launch": fetch + write,
           "note": "traffic = 2 x FETCH_SIZE + WRITE_SIZE per steady-state dispatch (gfx950 corrections)"}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 6:
        with open(sys.argv[6], "w") as fo:
            json.dump(out, fo, indent=1)


if __name__ == "__main__":
    main()
