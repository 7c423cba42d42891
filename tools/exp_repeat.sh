# Three default lines and three driver-shaped (20-step) lines back to back on one box. bash tools/exp_repeat.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0
for k in 1 2 3; do
  timeout -k 10 300 python bench.py > gpurun_out/r05x_bench_$k.json 2> gpurun_out/r05x_bench_$k.err || exit 1
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/r05x_bench20_$k.json 2> gpurun_out/r05x_bench20_$k.err || exit 1
done
python3 - <<'PY'
import json
for k in (1, 2, 3):
    d = json.loads(open(f"gpurun_out/r05x_bench_{k}.json").read().strip().splitlines()[-1])
    e = json.loads(open(f"gpurun_out/r05x_bench20_{k}.json").read().strip().splitlines()[-1])
    print(k, "default", round(d["value"] / 1e9, 3), "G", round(d["roofline"]["frac"], 3), "| 20-step", round(e["value"] / 1e9, 3), "G")
PY
