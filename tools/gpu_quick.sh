# Parity tests, then serialized and pipelined bench lines (development loop).
set -e
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
RMQ_DEBUG_SKIP=4 timeout -k 10 240 python bench.py --steps 300 --warmup 50 --no-cpu-baseline > gpurun_out/b_serial.log 2>&1
timeout -k 10 240 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/b_overlap.log 2>&1
