# Round-2 check: GPU parity tests, the driver's bench line (20 steps), a steady-state line
# (2000 steps), and rocprofv3 kernel-trace stats of the steady-state bench.
# usage: bash tools/gpu_r02.sh <tag> [extra bench args]
set -e
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=${1:-r02}; shift || true
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/${T}_bench20.json 2>gpurun_out/${T}_bench20.err
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/${T}_bench2000.json 2>gpurun_out/${T}_bench2000.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${T}_prof -o kt -- python3 $R/bench.py --no-cpu-baseline "$@" > $R/gpurun_out/${T}_bench_prof.log 2>&1
