# Fetch kernel check: the fetch GPU tests, a bench line with the fetch leg, and rocprofv3 kernel
# stats of the same command (fetch_kernel durations against the bench's event region).
# usage: bash tools/gpu_fetch2.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
T=$1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pinned.py tests/test_golden.py tests/test_tier.py tests/test_producer.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_fetch.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 400 --warmup 40 --no-cpu-baseline --host-steps 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${T}_kt -o kt -- python3 $R/bench.py --steps 400 --warmup 40 --no-cpu-baseline --host-steps 0 > $R/gpurun_out/${T}_kt.log 2>&1 || exit 1
