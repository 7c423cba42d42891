# A/B of the current library against variants/head: steady line (400 steps) and driver-shaped line
# (20 steps), N alternating pairs. usage: bash tools/gpu_ab.sh <tag> <pairs>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; N=${2:-2}
mkdir -p gpurun_out
Q="--no-cpu-baseline --fetch-rounds 0 --host-steps 0"
for rep in $(seq 1 $N); do
  for v in cur head; do
    if [ $v = cur ]; then L=$PWD/ripplemq_amd/libripplemq_engine.so; else L=$PWD/variants/head/libripplemq_engine.so; fi
    RMQ_LIB=$L timeout -k 10 200 python bench.py --steps 400 --warmup 40 $Q > gpurun_out/${T}_${v}_400_$rep.json 2>&1 || exit 1
    RMQ_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 $Q > gpurun_out/${T}_${v}_20_$rep.json 2>&1 || exit 1
  done
done
