#!/usr/bin/env python3
"""Summarise pipeline-launch phase stamps (RMQ_STAMPS=<csv>, one launch: RMQ_STAMPS_AT).

Rows: workgroup, wave, role (1 rank tiles, 2 column scans, 3 apply tasks, 4 partition threads),
t0..t7 s_memrealtime (100 MHz -> 10 ns). Stage 1/2 stamps are per workgroup (wave 0); stage 3 per
wave (stamps 2/3 bracket the wave's last task); partition threads per wave.
Prints, per stage, start/end spread relative to the first stamp of the launch and per-phase
percentiles."""
import sys

import numpy as np

PHASES = {
    1: ["loads+input scans", "radix passes", "seg scan+writes"],
    2: ["column scans+tile scan", "arrival + plan pass 1 (a destination)", "plan pass 2 (that destination)",
        "rest of the plan (transport)"],
    3: ["first task r1+tables+r2 issue", "(earlier tasks)", "last task finish", "(unused)",
        "(unused)", "(unused)"],
    4: ["(unused)", "(unused)", "(unused)", "(unused)", "(unused)", "partition apply + retention"],
}


def main(path):
    a = np.loadtxt(path, delimiter=",", skiprows=1, dtype=np.int64)
    t0 = a[:, 3][a[:, 3] > 0].min()
    print(f"{path}: launch span {(a[:, 3:][a[:, 3:] > 0].max() - t0) * 0.01:.2f} us")
    for stage, names in PHASES.items():
        r = a[a[:, 2] == stage]
        if stage in (1, 2):
            r = r[r[:, 1] == 0]
        if not len(r):
            continue
        raw = r[:, 3:3 + len(names) + 1]
        valid = (raw[:, 0] > 0) & (raw[:, -1] > 0)
        t = (raw[valid] - t0).astype(np.float64) * 0.01
        t[raw[valid] == 0] = np.nan
        if not len(t):
            continue
        print(f" stage {stage}: {len(t)} rows, start p0 {t[:, 0].min():.2f} p50 {np.median(t[:, 0]):.2f} "
              f"max {t[:, 0].max():.2f} | end p50 {np.median(t[:, -1]):.2f} max {t[:, -1].max():.2f} us")
        for k, n in enumerate(names):
            d = t[:, k + 1] - t[:, k]
            d = d[~np.isnan(d)]
            if not len(d):
                continue
            print(f"   {n:>26s}: p10 {np.percentile(d, 10):7.2f} p50 {np.percentile(d, 50):7.2f} "
                  f"p90 {np.percentile(d, 90):7.2f} max {d.max():7.2f} us")
    # steady plan events (PLAN_STAMP): wave i / 3's slot 5 + i % 3, relative to event 0
    names = ["start", "first scan done (totals in)", "scans and stores issued", "stores drained"]
    r = a[(a[:, 2] == 2) & (a[:, 1] == 0)]
    for wg in r[:, 0]:
        it = a[(a[:, 0] == wg) & (a[:, 2] == 2)]
        it = it[np.argsort(it[:, 1])]
        ev = [it[i // 3, 3 + 5 + i % 3] if i // 3 < len(it) else 0 for i in range(len(names))]
        if ev[0] > 0 and ev[-1] > 0 and it[0, 3 + 2] > 0:
            print("   steady plan: " + ", ".join(f"{n} {(t - ev[0]) * 0.01:.2f}" for n, t in zip(names, ev)) + " us")
    # the plan workgroup (stage 2 with a pass-1 stamp): wave w's slots 5..7 = pass-1 iteration w's
    # start, scan A done, stores drained
    r = a[(a[:, 2] == 2) & (a[:, 1] == 0) & (a[:, 5] > 0)]
    for wg in r[:, 0]:
        it = a[(a[:, 0] == wg) & (a[:, 2] == 2)]
        for row in it[np.argsort(it[:, 1])]:
            s5, s6, s7 = row[3 + 5], row[3 + 6], row[3 + 7]
            if s5 > 0:
                print(f"   plan pass-1 iteration {row[1]}: start {(s5 - t0) * 0.01:8.2f} us, to scan A "
                      f"{(s6 - s5) * 0.01:6.2f} us, to stores drained {(s7 - s5) * 0.01:6.2f} us")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)
