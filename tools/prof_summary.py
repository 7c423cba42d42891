#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (rocpd .db or kernel_trace.csv) as a per-kernel table.

usage: prof_summary.py <results.db | kernel_trace.csv> [name-filter]
Durations in microseconds (rocprofv3 records ns); one row per kernel name."""
import csv
import sqlite3
import statistics
import sys


def rows(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, s, e in c.execute("select name, start, end from kernels"):
            yield name, (e - s) / 1e3
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                yield r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3


def main():
    path = sys.argv[1]
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    by = {}
    for name, us in rows(path):
        if flt in name:
            by.setdefault(name, []).append(us)
    tot = sum(sum(v) for v in by.values()) or 1.0
    print(f"{'kernel':60s} {'calls':>7s} {'total_us':>12s} {'avg_us':>9s} {'med_us':>9s} {'min_us':>9s} {'max_us':>9s} {'pct':>6s}")
    for name, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        print(f"{name[:60]:60s} {len(v):7d} {sum(v):12.1f} {sum(v)/len(v):9.2f} {statistics.median(v):9.2f} "
              f"{min(v):9.2f} {max(v):9.2f} {100*sum(v)/tot:6.2f}")


if __name__ == "__main__":
    main()
