# Parity tests, ring-store alignment microbenchmark, default bench line with phase stamps.
set -e
R=$GRAFT_REPO_ROOT
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 120 ./tools/ring_align_bench > gpurun_out/ring_align.txt 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
RMQ_STAMPS=gpurun_out/st_g2.csv timeout -k 10 240 python bench.py --steps 200 --warmup 50 --no-cpu-baseline > gpurun_out/bs_g2.log 2>&1
python tools/stamps.py gpurun_out/st_g2.csv > gpurun_out/st_g2.txt
