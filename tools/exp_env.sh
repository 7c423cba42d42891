# A/B of an environment knob on one box: the GPU parity subset with the knob set, then alternating
# 400-step and 20-step lines without / with it. [EXTRA="bench args"] bash tools/exp_env.sh <tag> "<VAR=value ...>" [config]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1; E=$2; CF=${3:-B}
Q="--config $CF ${EXTRA:-} --no-cpu-baseline --fetch-rounds 0 --concurrent-rounds 0 --host-steps 0 --tier-rounds 0"
run() { local lim=$1 out=$2; shift 2; echo "[exp] $(date +%T) $out"; timeout -k 10 "$lim" "$@" > "gpurun_out/$out" 2> "gpurun_out/$out.err" || { echo "[exp] FAILED rc=$? $out"; tail -30 "gpurun_out/$out.err"; exit 1; }; }
run 900 "${T}_pytest.log" env $E python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "parity or golden or pipelined or config or large or world8 or replication"
tail -1 "gpurun_out/${T}_pytest.log"
for k in 1 2 3; do
  run 200 "${T}_off_${k}.json" python bench.py --steps 400 --warmup 40 $Q
  run 200 "${T}_on_${k}.json" env $E python bench.py --steps 400 --warmup 40 $Q
  run 200 "${T}_off20_${k}.json" python bench.py --steps 20 --warmup 5 $Q
  run 200 "${T}_on20_${k}.json" env $E python bench.py --steps 20 --warmup 5 $Q
done
python3 - gpurun_out/${T}_o*.json <<'PY'
import json, sys
for f in sorted(sys.argv[1:]):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], round(d["value"] / 1e9, 3), "G", round(d["roofline"]["mean_kernel_us"], 1), "us/launch")
PY
echo "[exp] $(date +%T) done"
