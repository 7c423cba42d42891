# Timing experiments: the default build with RMQ_DEBUG knobs (results invalid, timing only).
set -e
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for d in ${DBG:-0 16 31}; do
  RMQ_DEBUG=$d RMQ_STAMPS=gpurun_out/st_d$d.csv RMQ_STAMPS_AT=300 timeout -k 10 120 python bench.py --steps 400 --warmup 50 --no-cpu-baseline > gpurun_out/bst_d$d.log 2>&1 || true
  python tools/pipe_stamps.py gpurun_out/st_d$d.csv > gpurun_out/st_d$d.txt
  RMQ_DEBUG=$d timeout -k 10 120 python bench.py --steps 2000 --no-cpu-baseline > gpurun_out/b_d$d.log 2>&1 || true
done
