#!/usr/bin/env python3
"""Phase stamps of the role-split stage 3 (RMQ_S3_ROLES with RMQ_STAMPS): per loader / storer wave,
start, after the table barrier, first hand-off, end (storer: stores issued, then drained), and the
time each spent waiting (loader: for a free buffer; storer: for a published image). 10 ns ticks."""
import sys

import numpy as np


def pct(x):
    return f"p10 {np.percentile(x, 10):7.2f} p50 {np.percentile(x, 50):7.2f} p90 {np.percentile(x, 90):7.2f} max {x.max():7.2f}"


def main(path, loaders=3):
    a = np.loadtxt(path, delimiter=",", skiprows=1, dtype=np.int64)
    t0 = a[:, 3][a[:, 3] > 0].min()
    r = a[(a[:, 2] == 3) & (a[:, 3] > 0) & (a[:, 6] > 0)]
    print(f"{path}: launch span {(a[:, 3:][a[:, 3:] > 0].max() - t0) * 0.01:.2f} us, {len(r)} stage-3 waves")
    for name, sel in (("loader", r[:, 1] < loaders), ("storer", r[:, 1] >= loaders)):
        x = r[sel]
        if not len(x):
            continue
        t = (x[:, 3:9] - t0) * 0.01
        print(f" {name}s ({len(x)}):")
        print(f"   start               {pct(t[:, 0])}")
        print(f"   tables + barrier    {pct(t[:, 1] - t[:, 0])}")
        print(f"   to first hand-off   {pct(t[:, 2] - t[:, 1])}")
        print(f"   first hand-off->end {pct(t[:, 3] - t[:, 2])}")
        print(f"   end                 {pct(t[:, 3])}")
        print(f"   waiting (total)     {pct(x[:, 7] * 0.01)}")
        if name == "storer":
            print(f"   stores drained      {pct(t[:, 5])}")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)
