# Parity tests, then the default bench line twice (run-to-run spread) and the no-CRC-tables knob.
set -e
R=$GRAFT_REPO_ROOT
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
for k in a b; do
timeout -k 10 200 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/q_$k.json 2> gpurun_out/q_$k.err
done
RMQ_DEBUG=8 timeout -k 10 200 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/q_d8.json 2> gpurun_out/q_d8.err
