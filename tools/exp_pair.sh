set -o pipefail
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1
RMQ_S3_PAIR=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "parity or golden or pipelined or config" > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
bash tools/exp.sh $T - - RMQ_S3_PAIR=0 RMQ_S3_PAIR=1 RMQ_S3_PAIR=0 RMQ_S3_PAIR=1
Q="--no-cpu-baseline --fetch-rounds 0 --concurrent-rounds 0 --host-steps 0 --tier-rounds 0"
(cd /tmp && export TMPDIR=/tmp && RMQ_SPLIT=2 RMQ_S3_PAIR=1 timeout -s KILL 120 rocprofv3 --kernel-trace -f csv -d "$R/gpurun_out/${T}_kt2p" -o kt -- python3 "$R/bench.py" --steps 60 --warmup 10 $Q) > "$R/gpurun_out/${T}_kt2p.log" 2>&1 || exit 1
