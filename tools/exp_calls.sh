# Host timeline of fetch calls: tools/fetch_calls.py plain, then under rocprofv3 with the HIP API,
# kernel and copy traces. bash tools/exp_calls.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1
timeout -k 10 200 python tools/fetch_calls.py > gpurun_out/${T}_calls.json 2> gpurun_out/${T}_calls.err || { tail -20 gpurun_out/${T}_calls.err; exit 1; }
cat gpurun_out/${T}_calls.json
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace -f csv -d "$R/gpurun_out/${T}_ct" -o ct -- python3 "$R/tools/fetch_calls.py") > "$R/gpurun_out/${T}_ct.log" 2>&1 || { tail -20 "$R/gpurun_out/${T}_ct.log"; exit 1; }
ls gpurun_out/${T}_ct
