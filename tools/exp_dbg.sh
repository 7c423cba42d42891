# Timing-only RMQ_DEBUG lines of one config (results invalid; the lines are marked):
# bash tools/exp_dbg.sh <tag> <config> <bits...>   (1 no ring stores, 2 no CRC, 4 no payload loads, 8, 16)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1; CF=$2; shift 2
Q="--config $CF --no-cpu-baseline --fetch-rounds 0 --concurrent-rounds 0 --host-steps 0 --tier-rounds 0"
for d in 0 "$@"; do
  RMQ_DEBUG=$d timeout -k 10 200 python bench.py --steps 400 --warmup 40 $Q > gpurun_out/${T}_dbg$d.json 2> gpurun_out/${T}_dbg$d.err || { tail -20 gpurun_out/${T}_dbg$d.err; exit 1; }
done
python3 tools/show_lines.py gpurun_out/${T}_dbg*.json
