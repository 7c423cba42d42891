"""Summary of tools/gpu_abd.sh outputs: value and roofline fraction per variant, config and repeat."""
import glob
import json
import sys

tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/{tag}_*_*.json")):
    try:
        d = json.load(open(f))
    except ValueError:
        print(f, "unreadable")
        continue
    r = d["roofline"]
    print(f"{f}: {d['value'] / 1e9:.3f} G msgs/s frac {r['frac']:.3f} launch {r['mean_kernel_us']:.1f} us "
          f"bpl {r['batches_per_launch']:.2f}")
