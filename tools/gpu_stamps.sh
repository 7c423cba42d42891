# Phase stamps of one steady-state launch (launch 100) of the default bench, plus a DEBUG timing
# set: 1 no ring stores, 16 stage 3 alone. usage: bash tools/gpu_stamps.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1
mkdir -p gpurun_out
RMQ_STAMPS=gpurun_out/${T}_st.csv RMQ_STAMPS_AT=100 timeout -k 10 200 python bench.py --steps 600 --warmup 60 --no-cpu-baseline --fetch-rounds 0 --host-steps 0 > gpurun_out/${T}_stamped_B_1.json 2>&1 || exit 1
python tools/pipe_stamps.py gpurun_out/${T}_st.csv > gpurun_out/${T}_stamps.txt 2>&1
for d in 1 2 4 16; do
  RMQ_DEBUG=$d timeout -k 10 200 python bench.py --steps 400 --warmup 40 --no-cpu-baseline --fetch-rounds 0 --host-steps 0 > gpurun_out/${T}_dbg${d}_B_1.json 2>&1 || true
done
