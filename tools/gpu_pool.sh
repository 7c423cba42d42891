# Does input residency in the memory-side cache matter? Steady line with 48 / 8 / 2 distinct
# resident batches (48 x 7 MB exceeds the 256 MB MALL; 8 and 2 fit). usage: bash tools/gpu_pool.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1
mkdir -p gpurun_out
Q="--no-cpu-baseline --fetch-rounds 0 --host-steps 0"
for pool in 48 8 2 48; do
  timeout -k 10 200 python bench.py --steps 400 --warmup 40 --pool $pool $Q > gpurun_out/${T}_p${pool}_400_$RANDOM.json 2>&1 || exit 1
done
