# Bench the default library and experimental builds under build/*/ (RMQ_LIB), with phase stamps.
set -e
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for lib in ripplemq_amd/libripplemq_engine.so variants/*/libripplemq_engine.so; do
  tag=$(basename $(dirname $lib))
  RMQ_LIB=$PWD/$lib RMQ_STAMPS=gpurun_out/st_$tag.csv RMQ_STAMPS_AT=300 timeout -k 10 120 python bench.py --steps 400 --warmup 50 --no-cpu-baseline > gpurun_out/bst_$tag.log 2>&1
  python tools/pipe_stamps.py gpurun_out/st_$tag.csv > gpurun_out/st_$tag.txt
  RMQ_LIB=$PWD/$lib timeout -k 10 120 python bench.py --steps 2000 --no-cpu-baseline > gpurun_out/b_$tag.log 2>&1
done
