# Multi-rank rehearsal on one GPU: bench.py --transport local (ranks as threads, in-process
# transport), then the single-GPU line. usage: bash tools/gpu_repl_bench.sh <tag>
set -e
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=${1:-rb}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --gpus 2 --transport local --steps 200 --warmup 20 --segment-mb 2 --pool 8 --fetch-rounds 2 > gpurun_out/${T}_local2.json 2> gpurun_out/${T}_local2.err
timeout -k 10 300 python bench.py --gpus 4 --transport local --steps 100 --warmup 10 --segment-mb 1 --pool 4 --fetch-rounds 0 --config C > gpurun_out/${T}_local4.json 2> gpurun_out/${T}_local4.err
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_bench20.json 2>gpurun_out/${T}_bench20.err
