# rocprofv3 kernel stats of the bench with its fetch leg (few append steps).
set -e
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1; shift; R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${T}_prof -o kt -- python3 $R/bench.py --steps 100 --warmup 20 --no-cpu-baseline "$@" > $R/gpurun_out/${T}_bench.json 2>&1
