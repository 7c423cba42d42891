# Prefetch-role sweep (RMQ_PF_WGS): steady line (400 steps) and driver-shaped line (20 steps),
# two passes. usage: bash tools/gpu_pf.sh <tag> <wgs...>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; shift
mkdir -p gpurun_out
Q="--no-cpu-baseline --fetch-rounds 0 --host-steps 0"
for rep in 1 2; do
  for w in "$@"; do
    RMQ_PF_WGS=$w timeout -k 10 200 python bench.py --steps 400 --warmup 40 $Q > gpurun_out/${T}_pf${w}_400_$rep.json 2>&1 || exit 1
    RMQ_PF_WGS=$w timeout -k 10 200 python bench.py --steps 20 --warmup 5 $Q > gpurun_out/${T}_pf${w}_20_$rep.json 2>&1 || exit 1
  done
done
