# HIP API + kernel trace of the driver-shaped bench (--steps 20 --warmup 5): where the host time
# of the timed region goes (append calls, launches, the final synchronisation).
# usage: bash tools/gpu_hip20.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace -f csv -d $R/gpurun_out/${T}_ht -o ht -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --fetch-rounds 0 --host-steps 0 > $R/gpurun_out/${T}_b20.json 2>&1
