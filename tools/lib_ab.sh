# A/B of the current library against variants/NAME/ on any bench line (run through gpurun):
#   bash tools/lib_ab.sh <tag> <NAME> <bench.py args...>
# two pairs, each step under its own time limit; outputs gpurun_out/<tag>_{cur,NAME}_{1,2}.json
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1
V=$2
shift 2
mkdir -p gpurun_out
for k in 1 2; do
  for v in cur "$V"; do
    if [ "$v" = cur ]; then L=$GRAFT_REPO_ROOT/ripplemq_amd/libripplemq_engine.so; else L=$GRAFT_REPO_ROOT/variants/$V/libripplemq_engine.so; fi
    echo "[lib_ab] $(date +%T) $v $k"
    RMQ_LIB=$L timeout -k 10 200 python bench.py "$@" > "gpurun_out/${T}_${v}_$k.json" 2> "gpurun_out/${T}_${v}_$k.err" || { echo "[lib_ab] FAILED $v $k"; tail -5 "gpurun_out/${T}_${v}_$k.err"; exit 1; }
  done
done
echo "[lib_ab] done"
