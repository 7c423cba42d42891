# Parity tests, then a stamped bench run (phase times of launch 300) and the plain bench line.
set -e
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
RMQ_STAMPS=gpurun_out/st.csv RMQ_STAMPS_AT=300 timeout -k 10 240 python bench.py --steps 400 --warmup 50 --no-cpu-baseline > gpurun_out/b_st.log 2>&1
python tools/pipe_stamps.py gpurun_out/st.csv > gpurun_out/st.txt
timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1
