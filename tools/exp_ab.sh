# GPU parity subset, then A/B lines of one config: the current library against variants/<V>.
# bash tools/exp_ab.sh <tag> <V> <config> [pytest -k expr|-]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1; V=$2; CF=$3; K=${4:-"parity or golden or pipelined or config or large or world8"}
Q="--config $CF --no-cpu-baseline --fetch-rounds 0 --concurrent-rounds 0 --host-steps 0 --tier-rounds 0"
run() { local lim=$1 out=$2; shift 2; echo "[exp] $(date +%T) $out"; timeout -k 10 "$lim" "$@" > "gpurun_out/$out" 2> "gpurun_out/$out.err" || { echo "[exp] FAILED rc=$? $out"; tail -30 "gpurun_out/$out.err"; tail -30 "gpurun_out/$out"; exit 1; }; }
if [ "$K" != "-" ]; then run 900 "${T}_pytest.log" python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$K"; tail -1 "gpurun_out/${T}_pytest.log"; fi
for k in 1 2; do
  for v in cur $V; do
    if [ $v = cur ]; then L=$R/ripplemq_amd/libripplemq_engine.so; else L=$R/variants/$V/libripplemq_engine.so; fi
    RMQ_LIB=$L run 200 "${T}_${v}_${CF}_$k.json" python bench.py --steps 400 --warmup 40 $Q
  done
done
python3 tools/show_lines.py gpurun_out/${T}_*_${CF}_*.json
echo "[exp] $(date +%T) done"
