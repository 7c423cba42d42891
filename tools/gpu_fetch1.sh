# Fused fetch kernel check: the fetch GPU tests, then the whole GPU suite, the default bench line
# (fetch leg included), 20-step lines at groups 4/6/8 with RMQ_TRACE launch roles, and a rocprofv3
# kernel trace of the 20-step line. usage: bash tools/gpu_fetch1.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
T=$1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pinned.py tests/test_golden.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_fetch.txt 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --host-steps 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
for g in 4 6 8; do
  RMQ_TRACE=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --group $g --no-cpu-baseline --fetch-rounds 0 --host-steps 0 > gpurun_out/${T}_b20_g$g.json 2> gpurun_out/${T}_b20_g$g.err || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/${T}_kt20 -o kt -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --fetch-rounds 2 --host-steps 0 > $R/gpurun_out/${T}_kt20.log 2>&1 || exit 1
