# Stage-1 / stage-2 workgroup caps with stage 3 dispatched last (run through gpurun):
#   bash tools/caps_sweep.sh <tag> S1:S2 [S1:S2 ...]   (0 = no cap)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=$1; shift
Q="--no-cpu-baseline --fetch-rounds 0 --concurrent-rounds 0 --host-steps 0 --tier-rounds 0"
mkdir -p gpurun_out
for k in 1 2; do
  for c in "$@"; do
    s1=${c%%:*}; s2=${c##*:}
    env RMQ_S1_WGS=$s1 RMQ_S2_WGS=$s2 timeout -k 10 200 python bench.py --steps 400 --warmup 40 $Q > "gpurun_out/${T}_${s1}_${s2}_400_$k.json" 2>/dev/null || exit 1
    env RMQ_S1_WGS=$s1 RMQ_S2_WGS=$s2 timeout -k 10 200 python bench.py --steps 20 --warmup 5 $Q > "gpurun_out/${T}_${s1}_${s2}_20_$k.json" 2>/dev/null || exit 1
  done
done
echo "[caps_sweep] done"
