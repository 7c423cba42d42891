# Where the append launch's time goes (timing-only RMQ_DEBUG bits, never parity): steady line
# (400 steps) with 0 (reference), 1 (no ring stores), 2 (no CRC lookups), 4 (no payload loads),
# 8 (no CRC table copies), 16 (stages 1-2 skipped). usage: bash tools/gpu_dbg.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1
mkdir -p gpurun_out
Q="--steps 400 --warmup 40 --no-cpu-baseline --fetch-rounds 0 --host-steps 0"
for d in 0 1 2 4 8 16 0; do
  RMQ_DEBUG=$d timeout -k 10 200 python bench.py $Q > gpurun_out/${T}_dbg$d.json 2>&1
  rc=$?
  # a debug run may fail the bench's commit check (no stores): keep its line, stop on a crash
  if [ $rc -ge 124 ]; then exit $rc; fi
done
