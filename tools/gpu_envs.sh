# Phase stamps of one steady-state launch (launch 100) and the 1000-step bench line per engine
# environment. usage: bash tools/gpu_envs.sh <tag> "VAR=x VAR2=y" "VAR=z" ...
# (results with RMQ_DEBUG set are timing experiments only)
set -e
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1; shift
mkdir -p gpurun_out
n=0
for spec in "$@"; do
  n=$((n+1))
  echo "$spec" > gpurun_out/${T}_${n}_env.txt
  env $spec RMQ_STAMPS=gpurun_out/${T}_${n}_st.csv RMQ_STAMPS_AT=100 timeout -k 10 200 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline --fetch-rounds 0 > gpurun_out/${T}_${n}_b1000.json 2>&1
  python tools/pipe_stamps.py gpurun_out/${T}_${n}_st.csv > gpurun_out/${T}_${n}_stamps.txt
done
