#!/usr/bin/env python3
"""Per-launch and per-batch HBM traffic of one kernel from two rocprofv3 --pmc runs
(MI355X_MICROARCH.md "HBM").

usage: pmc_summary.py <FETCH_SIZE counter_collection.csv> <WRITE_SIZE counter_collection.csv>
                      <kernel substring> <group> <config> <streaming read bytes per batch> [out.json]

FETCH_SIZE / WRITE_SIZE are KiB per dispatch. On gfx950 FETCH_SIZE tallies the 128-B requests of
16-B-per-lane streaming reads at 64 B, so only those reads are undercounted by half: the corrected
read bytes add back half of the streaming share, which for the pipeline kernel is the payload that
stage 3 loads as aligned 16-byte blocks (`streaming read bytes per batch` x batches per launch).
Every other read of the kernel (pidx, len, rank words, histogram cells, partition state) is a 4- or
8-byte access and is taken as counted. WRITE_SIZE is exact for the 16-B stores. Only dispatches with
the modal grid size are averaged: the steady-state launches that carry every pipeline stage, each
with `group` batches."""
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
    fpath, wpath, flt, group, config, stream = sys.argv[1:7]
    G = int(group)
    gf, f = per_dispatch(fpath, "FETCH_SIZE", flt)
    gw, w = per_dispatch(wpath, "WRITE_SIZE", flt)
    raw, write = statistics.mean(f), statistics.mean(w)
    corr = raw + 0.5 * float(stream) * G
    out = {"kernel": flt, "group": G, "config": config, "grid_size": [gf, gw],
           "dispatches": [len(f), len(w)],
           "fetch_size_raw_bytes_per_launch": raw, "fetch_bytes_per_launch": corr,
           "write_bytes_per_launch": write, "traffic_bytes_per_launch": corr + write,
           "traffic_bytes_per_batch": (corr + write) / G, "traffic_raw_bytes_per_batch": (raw + write) / G,
           "streaming_read_bytes_per_batch": float(stream),
           "note": "per launch of `group` batches; fetch = FETCH_SIZE + half the 16-B streaming reads "
                   "(gfx950 counts those at 64 of 128 B); write = WRITE_SIZE"}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 7:
        with open(sys.argv[7], "w") as fo:
            json.dump(out, fo, indent=1)


if __name__ == "__main__":
    main()
