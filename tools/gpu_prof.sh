# rocprofv3 kernel trace + stats of the default bench line, then PMC passes for HBM traffic
# (FETCH_SIZE and WRITE_SIZE in separate passes, MI355X_MICROARCH.md "HBM").
set -e
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof -o kt -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench_prof.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $R/gpurun_out/pmc_fetch -o pf -- python3 $R/bench.py --steps 300 --warmup 50 --no-cpu-baseline > $R/gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/gpurun_out/pmc_write -o pw -- python3 $R/bench.py --steps 300 --warmup 50 --no-cpu-baseline > $R/gpurun_out/pmc_write.log 2>&1
