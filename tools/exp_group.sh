# Launch-group size sweep of the driver-shaped (20-step) and steady (600-step) lines, then the
# 2-rank rehearsal (local transport) and its kernel trace. bash tools/exp_group.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1
Q="--no-cpu-baseline --fetch-rounds 0 --concurrent-rounds 0 --host-steps 0 --tier-rounds 0"
run() { local lim=$1 out=$2; shift 2; echo "[exp] $(date +%T) $out"; timeout -k 10 "$lim" "$@" > "gpurun_out/$out" 2> "gpurun_out/$out.err" || { echo "[exp] FAILED rc=$? $out"; tail -30 "gpurun_out/$out.err"; exit 1; }; }
for k in 1 2; do
  for g in 4 5 6 8; do
    run 200 "${T}_g${g}_20_$k.json" python bench.py --steps 20 --warmup 8 --group $g $Q
    run 200 "${T}_g${g}_600_$k.json" python bench.py --steps 600 --warmup 60 --group $g $Q
  done
done
python tools/show_lines.py gpurun_out/${T}_g*.json
run 300 "${T}_local2.json" python bench.py --gpus 2 --transport local --steps 200 --warmup 20 --segment-mb 2 --pool 8 $Q
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/${T}_l2kt" -o kt -- python3 "$R/bench.py" --gpus 2 --transport local --steps 200 --warmup 20 --segment-mb 2 --pool 8 $Q) > "$R/gpurun_out/${T}_l2kt.log" 2>&1 || exit 1
python3 - "$R/gpurun_out/${T}_local2.json" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("local2", d["value"]/1e9, "G", d["xgmi"]["host_waits_for_round_sizes"], d["xgmi"]["host_wait_ms"], d["ms_per_step"])
PY
echo "[exp] $(date +%T) done"
