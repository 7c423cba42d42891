# Config D bench lines under several RMQ_BIG_WGS values. usage: bash tools/gpu_envd.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1
mkdir -p gpurun_out
for w in 128 256 512 1024 2048; do
  RMQ_BIG_WGS=$w timeout -k 10 200 python bench.py --config D --pool 16 --steps 100 --warmup 10 --no-cpu-baseline --fetch-rounds 0 --host-steps 0 > gpurun_out/${T}_w${w}_D_1.json 2>&1 || exit 1
done
RMQ_BIG_WGS=512 timeout -k 10 200 python bench.py --steps 400 --warmup 40 --no-cpu-baseline --fetch-rounds 0 --host-steps 0 > gpurun_out/${T}_w512_B_1.json 2>&1 || exit 1
RMQ_BIG_WGS=64 timeout -k 10 200 python bench.py --steps 400 --warmup 40 --no-cpu-baseline --fetch-rounds 0 --host-steps 0 > gpurun_out/${T}_w64_B_1.json 2>&1
