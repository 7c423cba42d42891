# Round-2 measurement set: multi-rank rehearsal on one GPU (local transport), rocprofv3 kernel stats
# of the default bench, PMC traffic passes (separate), the driver-shaped and the default bench line.
set -e
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=${1:-r02s}; R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --gpus 2 --transport local --steps 200 --warmup 20 --segment-mb 2 --pool 8 --fetch-rounds 2 > gpurun_out/${T}_local2.json 2> gpurun_out/${T}_local2.err
timeout -k 10 300 python bench.py --gpus 4 --transport local --steps 100 --warmup 10 --segment-mb 1 --pool 4 --fetch-rounds 0 --config C > gpurun_out/${T}_local4.json 2> gpurun_out/${T}_local4.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${T}_prof -o kt -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/${T}_bench_prof.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $R/gpurun_out/${T}_pmc_fetch -o pf -- python3 $R/bench.py --steps 300 --warmup 50 --no-cpu-baseline --fetch-rounds 0 > $R/gpurun_out/${T}_pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/gpurun_out/${T}_pmc_write -o pw -- python3 $R/bench.py --steps 300 --warmup 50 --no-cpu-baseline --fetch-rounds 0 > $R/gpurun_out/${T}_pmc_write.log 2>&1
cd $R
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench20.json 2> gpurun_out/${T}_bench20.err
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
