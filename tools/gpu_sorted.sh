# Parity tests, then stage 3 in partition-sorted order (default) vs input order (RMQ_DEBUG=32).
set -e
R=$GRAFT_REPO_ROOT
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
for g in 2 4; do for d in 0 32; do
RMQ_DEBUG=$d timeout -k 10 200 python bench.py --group $g --no-cpu-baseline > gpurun_out/srt_${d}_g$g.json 2> gpurun_out/srt_${d}_g$g.err
done; done
RMQ_STAMPS=gpurun_out/st_srt_g4.csv timeout -k 10 240 python bench.py --steps 200 --warmup 50 --no-cpu-baseline > gpurun_out/bs_srt_g4.log 2>&1
