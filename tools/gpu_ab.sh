# GPU parity tests (default settings; NOTEST=1 skips them), then per engine environment the
# driver-shaped bench line (20 steps) and a 1000-step line with phase stamps of launch 100.
# usage: bash tools/gpu_ab.sh <tag> "VAR=x ..." ...
set -e
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1; shift
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
fi
n=0
for spec in "$@"; do
  n=$((n+1))
  echo "$spec" > gpurun_out/${T}_${n}_env.txt
  env $spec timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --fetch-rounds 0 > gpurun_out/${T}_${n}_b20.json 2>&1
  env $spec RMQ_STAMPS=gpurun_out/${T}_${n}_st.csv RMQ_STAMPS_AT=100 timeout -k 10 200 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline --fetch-rounds 0 > gpurun_out/${T}_${n}_b1000.json 2>&1
  python tools/pipe_stamps.py gpurun_out/${T}_${n}_st.csv > gpurun_out/${T}_${n}_stamps.txt
done
