# Bench line (default group) + rocprofv3 kernel stats + PMC passes + phase stamps at groups 1 and 2.
set -e
R=$GRAFT_REPO_ROOT
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
for g in 1 2; do RMQ_STAMPS=$R/gpurun_out/stamps_g$g.csv RMQ_STAMPS_AT=300 timeout -k 10 200 python bench.py --group $g --steps 800 --warmup 100 --no-cpu-baseline > gpurun_out/bench_stamps_g$g.json 2>&1; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof -o kt -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench_prof.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $R/gpurun_out/pmc_fetch -o pf -- python3 $R/bench.py --steps 300 --warmup 50 --no-cpu-baseline > $R/gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/gpurun_out/pmc_write -o pw -- python3 $R/bench.py --steps 300 --warmup 50 --no-cpu-baseline > $R/gpurun_out/pmc_write.log 2>&1
