"""Summary of tools/gpu_sweep.sh outputs."""
import glob
import json
import os
import sys

tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/{tag}_s*_B_1.json"), key=lambda x: int(x.split("_s")[-1].split("_")[0])):
    env = open(f.replace("_B_1.json", "_env.txt")).read().strip() if os.path.exists(f.replace("_B_1.json", "_env.txt")) else ""
    try:
        d = json.load(open(f))
    except ValueError:
        print(f, env, "unreadable")
        continue
    r = d["roofline"]
    print(f"{env:40s} {d['value'] / 1e9:.3f} G frac {r['frac']:.3f} launch {r['mean_kernel_us']:.1f} us")
