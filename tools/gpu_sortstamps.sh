set -e
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
RMQ_DEBUG_SKIP=4 RMQ_STAMPS=gpurun_out/ss.csv timeout -k 10 240 python bench.py --steps 200 --warmup 50 --no-cpu-baseline > gpurun_out/bss.log 2>&1
python tools/stamps.py gpurun_out/ss.csv.sort.csv gpurun_out/ss.csv > gpurun_out/ss.txt
