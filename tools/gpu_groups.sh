# Parity tests, then the bench line per launch-group size, and phase stamps of one group-8 launch.
set -e
R=$GRAFT_REPO_ROOT
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
for g in 4 6 8; do
timeout -k 10 200 python bench.py --group $g --no-cpu-baseline > gpurun_out/grp_g$g.json 2> gpurun_out/grp_g$g.err
done
RMQ_STAMPS_AT=20 RMQ_STAMPS=gpurun_out/st_g8.csv timeout -k 10 240 python bench.py --group 8 --steps 200 --warmup 50 --no-cpu-baseline > gpurun_out/bs_g8.log 2>&1
RMQ_STAMPS_AT=30 RMQ_STAMPS=gpurun_out/st_g4.csv timeout -k 10 240 python bench.py --group 4 --steps 200 --warmup 50 --no-cpu-baseline > gpurun_out/bs_g4.log 2>&1
