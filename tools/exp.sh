# Ad-hoc experiment driver (run through gpurun): GPU parity subset, then A/B lines.
#   bash tools/exp.sh <tag> <pytest -k expr|-> <ab variant|-> [KNOB=val ...]
# every step under its own time limit; the script stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1; K=$2; V=$3; shift 3
mkdir -p gpurun_out
Q="--no-cpu-baseline --fetch-rounds 0 --concurrent-rounds 0 --host-steps 0 --tier-rounds 0"
run() { local lim=$1 out=$2; shift 2; echo "[exp] $(date +%T) $out"; timeout -k 10 "$lim" "$@" > "gpurun_out/$out" 2> "gpurun_out/$out.err" || { echo "[exp] FAILED rc=$? $out"; tail -30 "gpurun_out/$out.err"; tail -30 "gpurun_out/$out"; exit 1; }; }
if [ "$K" != "-" ]; then run 900 "${T}_pytest.log" python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$K"; fi
if [ "$V" != "-" ]; then
  for k in 1 2; do
    for v in cur $V; do
      if [ $v = cur ]; then L=$GRAFT_REPO_ROOT/ripplemq_amd/libripplemq_engine.so; else L=$GRAFT_REPO_ROOT/variants/$V/libripplemq_engine.so; fi
      RMQ_LIB=$L run 200 "${T}_${v}_600_$k.json" python bench.py --steps 600 --warmup 60 $Q
      RMQ_LIB=$L run 200 "${T}_${v}_20_$k.json" python bench.py --steps 20 --warmup 5 $Q
    done
  done
fi
for kv in "$@"; do
  env "$kv" timeout -k 10 200 python bench.py --steps 600 --warmup 60 $Q > "gpurun_out/${T}_${kv}_600.json" 2> "gpurun_out/${T}_${kv}_600.err" || { echo "[exp] FAILED $kv"; tail -5 "gpurun_out/${T}_${kv}_600.err"; exit 1; }
  env "$kv" timeout -k 10 200 python bench.py --steps 20 --warmup 5 $Q > "gpurun_out/${T}_${kv}_20.json" 2> "gpurun_out/${T}_${kv}_20.err" || { echo "[exp] FAILED $kv"; exit 1; }
done
python tools/show_lines.py gpurun_out/${T}_*.json 2>/dev/null || true
echo "[exp] $(date +%T) done"
