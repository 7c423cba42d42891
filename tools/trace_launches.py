#!/usr/bin/env python3
"""Per-launch timeline of the pipeline kernel from a rocprofv3 kernel trace (kt_kernel_trace.csv):
start (relative to the first pipeline launch), duration and gap before it, plus the other kernels."""
import csv
import sys


def main(path, last=20):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    pipe = [r for r in rows if "pipeline_kernel" in r["Kernel_Name"]]
    if not pipe:
        print(path, "no pipeline launches")
        return
    t0 = int(pipe[0]["Start_Timestamp"])
    print(f"{path}: {len(pipe)} pipeline launches")
    prev_end = None
    for r in pipe[-last:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1e3 if prev_end else float("nan")
        print(f"  t={(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:7.1f} us  gap {gap:6.1f} us  grid {r.get('Grid_Size_X', r.get('Grid_Size', ''))}")
        prev_end = e


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)
