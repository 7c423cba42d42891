# Config B bench lines under environment settings given as arguments ("VAR=v VAR2=w" each).
# usage: bash tools/gpu_sweep.sh <tag> "<env1>" "<env2>" ...
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; shift
mkdir -p gpurun_out
k=0
for e in "$@"; do
  k=$((k + 1))
  echo "$e" > gpurun_out/${T}_s${k}_env.txt
  env $e timeout -k 10 200 python bench.py --steps 600 --warmup 60 --no-cpu-baseline --fetch-rounds 0 --host-steps 0 > gpurun_out/${T}_s${k}_B_1.json 2>&1 || exit 1
done
