# parity subset, then A/B of the current library against variants/$2 (600- and 20-step lines, two
# pairs), then apply-alone kernel traces (RMQ_SPLIT=2) of both. bash tools/exp2.sh <tag> <variant> [-k expr]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1; V=$2; K=${3:-"parity or golden or pipelined or config"}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
bash tools/exp.sh $T - $V || exit 1
Q="--no-cpu-baseline --fetch-rounds 0 --concurrent-rounds 0 --host-steps 0 --tier-rounds 0"
for v in cur $V; do
  if [ $v = cur ]; then L=$R/ripplemq_amd/libripplemq_engine.so; else L=$R/variants/$V/libripplemq_engine.so; fi
  (cd /tmp && export TMPDIR=/tmp && RMQ_LIB=$L RMQ_SPLIT=2 timeout -s KILL 120 rocprofv3 --kernel-trace -f csv -d "$R/gpurun_out/${T}_kt_$v" -o kt -- python3 "$R/bench.py" --steps 60 --warmup 10 $Q) > "$R/gpurun_out/${T}_kt_$v.log" 2>&1 || exit 1
done
python3 tools/kt_apply.py gpurun_out/${T}_kt_cur gpurun_out/${T}_kt_$V
