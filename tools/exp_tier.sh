# The tier leg alone (and the tier GPU test), twice. bash tools/exp_tier.sh <tag>
# (round 5's chunked-spill sweep set RMQ_TIER_CHUNKS per run, CHUNKS="1 2 4 8"; the chunked spill was reverted)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1
timeout -k 10 300 python -u -m pytest tests/test_tier.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/${T}_tiertest.log 2>&1 || { tail -30 gpurun_out/${T}_tiertest.log; exit 1; }
tail -1 gpurun_out/${T}_tiertest.log
for k in 1 2; do
  for ch in ${CHUNKS:-4}; do
    RMQ_TIER_CHUNKS=$ch timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --host-steps 0 --fetch-rounds 0 --concurrent-rounds 0 --tier-rounds 20 > gpurun_out/${T}_tier_c${ch}_$k.json 2> gpurun_out/${T}_tier_c${ch}_$k.err || { tail -30 gpurun_out/${T}_tier_c${ch}_$k.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${T}_tier_c${ch}_$k.json').read().strip().splitlines()[-1]); print('chunks $ch', json.dumps(d['tier']['spill']))"
  done
done
# diagnosis only (not durable): the same leg with the files in /dev/shm
if [ -n "$SHM" ]; then
  RMQ_TIER_DIR=/dev/shm timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --host-steps 0 --fetch-rounds 0 --concurrent-rounds 0 --tier-rounds 20 > gpurun_out/${T}_tier_shm.json 2> gpurun_out/${T}_tier_shm.err || { tail -30 gpurun_out/${T}_tier_shm.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${T}_tier_shm.json').read().strip().splitlines()[-1]); print('shm', json.dumps(d['tier']['spill']))"
  df -h /tmp /dev/shm | cat
fi
