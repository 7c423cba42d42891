#!/usr/bin/env python3
"""Per-kernel duration summary of a rocprofv3 kernel trace (kt_kernel_trace.csv), in dispatch order.

  python tools/kernel_trace.py <trace.csv> [name-substring ...] [--groups N]

Prints, for every kernel whose name contains one of the substrings (all kernels if none), the
mean duration of each run of N consecutive dispatches (default 10: the bench's fetch legs are 10
rounds of max = 10, then 10 of max = 1024)."""
import csv
import sys


def main(argv):
    n = 10
    if "--groups" in argv:
        i = argv.index("--groups")
        n = int(argv[i + 1])
        argv = argv[:i] + argv[i + 2:]
    path, subs = argv[0], argv[1:]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    by = {}
    for r in rows:
        name = r["Kernel_Name"]
        if subs and not any(s in name for s in subs):
            continue
        by.setdefault(name, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    for name, d in by.items():
        runs = [sum(d[i:i + n]) / len(d[i:i + n]) for i in range(0, len(d), n)]
        print(f"{name[:60]:60s} {len(d):5d} calls; mean us per run of {n}: " + " ".join(f"{x:.1f}" for x in runs[:12]))


if __name__ == "__main__":
    main(sys.argv[1:])
