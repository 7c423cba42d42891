# Per-launch durations around the timed region: warmup 5 vs 100 vs 100 + an idle host gap.
set -e
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1; R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/${T}_w5_kt -o kt -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --fetch-rounds 0 > $R/gpurun_out/${T}_w5.json 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/${T}_w100_kt -o kt -- python3 $R/bench.py --steps 20 --warmup 100 --no-cpu-baseline --fetch-rounds 0 > $R/gpurun_out/${T}_w100.json 2>&1
RMQ_BENCH_IDLE_MS=200 timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/${T}_w100i_kt -o kt -- python3 $R/bench.py --steps 20 --warmup 100 --no-cpu-baseline --fetch-rounds 0 > $R/gpurun_out/${T}_w100i.json 2>&1
