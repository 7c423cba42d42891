# Input pool layout: an allocation per array vs one region (steady and 20-step lines, 2 passes).
# usage: bash tools/gpu_inputs.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1
mkdir -p gpurun_out
Q="--no-cpu-baseline --fetch-rounds 0 --host-steps 0"
for rep in 1 2; do
  for m in arrays region; do
    timeout -k 10 200 python bench.py --steps 400 --warmup 40 --inputs $m $Q > gpurun_out/${T}_${m}_400_$rep.json 2>&1 || exit 1
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --inputs $m $Q > gpurun_out/${T}_${m}_20_$rep.json 2>&1 || exit 1
  done
done
timeout -k 10 200 python bench.py --steps 400 --warmup 40 --inputs region --pool 8 $Q > gpurun_out/${T}_regionp8_400_1.json 2>&1
