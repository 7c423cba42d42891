set -e
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
RMQ_DEBUG_SKIP=4 RMQ_STAMPS=gpurun_out/stamps_serial.csv timeout -k 10 240 python bench.py --steps 200 --warmup 50 --no-cpu-baseline > gpurun_out/b_serial.log 2>&1
RMQ_STAMPS=gpurun_out/stamps_overlap.csv timeout -k 10 240 python bench.py --steps 200 --warmup 50 --no-cpu-baseline > gpurun_out/b_overlap.log 2>&1
python tools/stamps.py gpurun_out/stamps_serial.csv gpurun_out/stamps_overlap.csv > gpurun_out/stamps.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o r1 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 500 --warmup 100 > $GRAFT_REPO_ROOT/gpurun_out/b_prof.log 2>&1
