# Per-launch durations of the driver-shaped bench (20 steps, 5 warmup) and the 1000-step line by ring size.
set -e
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1; shift; R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for mb in "$@"; do
  timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/${T}_s${mb}_kt -o kt -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --fetch-rounds 0 --segment-mb $mb > $R/gpurun_out/${T}_s${mb}_b20.json 2>&1
  timeout -k 10 200 python3 $R/bench.py --steps 1000 --warmup 100 --no-cpu-baseline --fetch-rounds 0 --segment-mb $mb > $R/gpurun_out/${T}_s${mb}_b1000.json 2>&1
done
