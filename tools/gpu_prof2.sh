# Round profile of the default bench line: parity tests, bench (with CPU baseline), rocprofv3
# kernel trace + stats, and the FETCH_SIZE / WRITE_SIZE PMC passes (separate runs).
set -e
R=$GRAFT_REPO_ROOT
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof -o kt -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench_prof.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $R/gpurun_out/pmc_fetch -o pf -- python3 $R/bench.py --steps 300 --warmup 50 --no-cpu-baseline > $R/gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/gpurun_out/pmc_write -o pw -- python3 $R/bench.py --steps 300 --warmup 50 --no-cpu-baseline > $R/gpurun_out/pmc_write.log 2>&1
cd $R
RMQ_STAMPS_AT=30 RMQ_STAMPS=gpurun_out/st_g4.csv timeout -k 10 240 python bench.py --steps 200 --warmup 50 --no-cpu-baseline > gpurun_out/bs_g4.log 2>&1
