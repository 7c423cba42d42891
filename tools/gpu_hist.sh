# Steady line of earlier commits (each with its own bench.py, built under variants/wt_<commit>)
# against the current tree, equal rings (16 MiB: round 1's whole-batch space rule needs them),
# two passes. usage: bash tools/gpu_hist.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT; T=$1
mkdir -p gpurun_out
for rep in 1 2; do
  (cd variants/wt_0a6681b && timeout -k 10 200 python bench.py --steps 400 --warmup 40 --no-cpu-baseline --segment-mb 16) > gpurun_out/${T}_r1_400_$rep.json 2>&1 || exit 1
  (cd variants/wt_c4f3a2c && timeout -k 10 200 python bench.py --steps 400 --warmup 40 --no-cpu-baseline --segment-mb 16 --fetch-rounds 0) > gpurun_out/${T}_c4f_400_$rep.json 2>&1 || exit 1
  (cd variants/wt_f00a66a && timeout -k 10 200 python bench.py --steps 400 --warmup 40 --no-cpu-baseline --segment-mb 16 --fetch-rounds 0) > gpurun_out/${T}_f00_400_$rep.json 2>&1 || exit 1
  timeout -k 10 200 python bench.py --steps 400 --warmup 40 --no-cpu-baseline --rings equal --segment-mb 16 --fetch-rounds 0 --host-steps 0 > gpurun_out/${T}_cur_400_$rep.json 2>&1 || exit 1
done
