#!/usr/bin/env python3
"""One row per bench JSON line: msgs/s, roofline fraction, mean launch, batches per launch."""
import json
import sys

for path in sys.argv[1:]:
    try:
        txt = [l for l in open(path) if l.startswith("{")]
        d = json.loads(txt[-1])
    except (OSError, IndexError, ValueError) as ex:
        print(f"{path:50s} unreadable ({ex.__class__.__name__})")
        continue
    r = d["roofline"]
    print(f"{path:50s} {d['value'] / 1e9:6.3f} G  frac {r['frac']:.3f}  {r['mean_kernel_us']:6.1f} us/launch  "
          f"{r['batches_per_launch']:.2f} b/l")
