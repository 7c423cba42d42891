# Stage-3 wave count: looping waves (default) vs one wave per task (RMQ_WG3_ALL=1), groups 1-4.
set -e
R=$GRAFT_REPO_ROOT
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for a in 0 1; do for g in 1 2 3 4; do
RMQ_WG3_ALL=$a timeout -k 10 200 python bench.py --group $g --no-cpu-baseline > gpurun_out/wg3_${a}_g$g.json 2> gpurun_out/wg3_${a}_g$g.err
done; done
RMQ_WG3_ALL=1 RMQ_STAMPS=gpurun_out/st_all_g2.csv timeout -k 10 240 python bench.py --steps 200 --warmup 50 --no-cpu-baseline > gpurun_out/bs_all_g2.log 2>&1
RMQ_WG3_ALL=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1
