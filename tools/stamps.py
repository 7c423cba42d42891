"""Summarise the append kernel's per-phase stamps (RMQ_STAMPS=<csv> diagnostic run).

s_memrealtime ticks at 100 MHz on gfx950 (10 ns). Prints per-phase percentiles over tiles and
the launch span (first stamp 0 .. last stamp 7)."""
import sys

import numpy as np

NAMES = ["loads+dma issue+state", "scan/publish+dma wait", "crc", "look-back",
         "offsets/index/headers", "ring stores", "finalize+stats"]


def main(path):
    a = np.loadtxt(path, delimiter=",", skiprows=1, dtype=np.int64)
    t = a[:, 1:].astype(np.float64) * 10e-3  # µs
    t0 = t[:, 0].min()
    print(f"{path}: tiles={len(t)} span={t[:, 7].max() - t0:.2f} us, "
          f"start spread p50={np.percentile(t[:, 0] - t0, 50):.2f} max={(t[:, 0] - t0).max():.2f} us")
    for k in range(7):
        d = t[:, k + 1] - t[:, k]
        print(f"  {NAMES[k]:>24s}: p10 {np.percentile(d, 10):7.2f}  p50 {np.percentile(d, 50):7.2f}  "
              f"p90 {np.percentile(d, 90):7.2f}  max {d.max():7.2f} us")
    e = t[:, 7] - t0
    print(f"  {'tile end':>24s}: p10 {np.percentile(e, 10):7.2f}  p50 {np.percentile(e, 50):7.2f}  "
          f"p90 {np.percentile(e, 90):7.2f}  max {e.max():7.2f} us")




SORT_NAMES = ["loads", "first-pass byte scan", "ranking", "hist publish", "digit sweep",
              "byte sums + block scan", "scatter"]


def main_sort(path):
    a = np.loadtxt(path, delimiter=",", skiprows=1, dtype=np.int64)
    base = a[:, 2:].min()
    for k in sorted(set(a[:, 0].tolist())):
        r = a[a[:, 0] == k]
        t = (r[:, 2:] - base).astype(np.float64) * 10e-3
        print(f"{path} pass {k}: tiles={len(r)} start min {t[:, 0].min():.2f} max {t[:, 0].max():.2f}  "
              f"end max {t[:, 7].max():.2f} us")
        for q in range(7):
            d = t[:, q + 1] - t[:, q]
            print(f"  {SORT_NAMES[q]:>24s}: p10 {np.percentile(d, 10):7.2f}  p50 {np.percentile(d, 50):7.2f}  "
                  f"p90 {np.percentile(d, 90):7.2f}  max {d.max():7.2f} us")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        (main_sort if p.endswith(".sort.csv") else main)(p)
