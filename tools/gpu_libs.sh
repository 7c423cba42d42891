# 20-step and 1000-step (phase stamps of launch 100) bench lines for the default library and each
# variants/*/ build (RMQ_LIB). usage: bash tools/gpu_libs.sh <tag>   (then tools/show_envs.sh <tag>)
set -e
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1
mkdir -p gpurun_out
for lib in ripplemq_amd/libripplemq_engine.so variants/*/libripplemq_engine.so; do
  v=$(basename $(dirname $lib))
  echo "RMQ_LIB=$lib" > gpurun_out/${T}_${v}_env.txt
  RMQ_LIB=$PWD/$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --fetch-rounds 0 > gpurun_out/${T}_${v}_b20.json 2>&1
  RMQ_LIB=$PWD/$lib RMQ_STAMPS=gpurun_out/${T}_${v}_st.csv RMQ_STAMPS_AT=100 timeout -k 10 200 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline --fetch-rounds 0 > gpurun_out/${T}_${v}_b1000.json 2>&1
  python tools/pipe_stamps.py gpurun_out/${T}_${v}_st.csv > gpurun_out/${T}_${v}_stamps.txt
done
