# GPU parity tests only (optionally a -k expression): bash tools/gpu_tests.sh <tag> [-k expr]
set -e
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=${1:-t}; shift || true
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "$@" > gpurun_out/${T}_pytest_gpu.log 2>&1
