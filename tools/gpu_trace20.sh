# Kernel trace of the driver-shaped bench (20 steps, 5 warmup) for the default library and each
# variants/*/ build: per-launch pipeline durations. usage: bash tools/gpu_trace20.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1; R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
LIBS=$(ls ripplemq_amd/libripplemq_engine.so variants/*/libripplemq_engine.so 2>/dev/null)
cd /tmp && export TMPDIR=/tmp
for lib in $LIBS; do
  v=$(basename $(dirname $lib))
  RMQ_LIB=$R/$lib timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/${T}_${v}_kt -o kt -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --fetch-rounds 0 > $R/gpurun_out/${T}_${v}_b20.json 2>&1
done
