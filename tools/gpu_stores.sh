set -e
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for f in ${FLAGS:-0 4 8}; do
RMQ_DEBUG_FLAGS=$f RMQ_STAMPS=gpurun_out/st_$f.csv timeout -k 10 240 python bench.py --steps 200 --warmup 50 --no-cpu-baseline > gpurun_out/bs_$f.log 2>&1
python tools/stamps.py gpurun_out/st_$f.csv > gpurun_out/st_$f.txt
done
