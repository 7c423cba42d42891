# Config D (records of 64 B - 16 KB, RF 5): the line, per-wave phase stamps of one launch, the
# apply kernel alone (RMQ_SPLIT=2) in a kernel trace, and the HBM traffic (separate PMC passes).
# bash tools/exp_D.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1
Q="--config D --no-cpu-baseline --fetch-rounds 0 --concurrent-rounds 0 --host-steps 0 --tier-rounds 0"
run() { local lim=$1 out=$2; shift 2; echo "[exp] $(date +%T) $out"; timeout -k 10 "$lim" "$@" > "gpurun_out/$out" 2> "gpurun_out/$out.err" || { echo "[exp] FAILED rc=$? $out"; tail -30 "gpurun_out/$out.err"; exit 1; }; }
run 200 "${T}_D.json" python bench.py --steps 400 --warmup 40 $Q
python3 tools/show_lines.py gpurun_out/${T}_D.json
RMQ_STAMPS=gpurun_out/${T}_Dst.csv RMQ_STAMPS_AT=60 run 200 "${T}_Dstamped.json" python bench.py --steps 200 --warmup 40 $Q
python tools/pipe_stamps.py "gpurun_out/${T}_Dst.csv" > "gpurun_out/${T}_Dstamps.txt" 2>&1 || true
(cd /tmp && export TMPDIR=/tmp && RMQ_SPLIT=2 timeout -s KILL 120 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/${T}_Dkt" -o kt -- python3 "$R/bench.py" --steps 200 --warmup 20 $Q) > "$R/gpurun_out/${T}_Dkt.log" 2>&1 || exit 1
python3 tools/kt_apply.py gpurun_out/${T}_Dkt
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -f csv -d "$R/gpurun_out/${T}_Dpf" -o pf -- python3 "$R/bench.py" --steps 200 --warmup 20 $Q) > "$R/gpurun_out/${T}_Dpf.log" 2>&1 || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -f csv -d "$R/gpurun_out/${T}_Dpw" -o pw -- python3 "$R/bench.py" --steps 200 --warmup 20 $Q) > "$R/gpurun_out/${T}_Dpw.log" 2>&1 || exit 1
ls gpurun_out/${T}_Dpf gpurun_out/${T}_Dpw
echo "[exp] $(date +%T) done"
