# A/B of the current library against variants/t512 on the replication path: 2 ranks on one GPU over
# the in-process transport (config B, 2 pairs; config D, 1 pair). usage: bash tools/gpu_local_ab.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1
mkdir -p gpurun_out
Q="--no-cpu-baseline --fetch-rounds 0 --host-steps 0 --gpus 2 --transport local"
lib() { if [ $1 = cur ]; then echo $PWD/ripplemq_amd/libripplemq_engine.so; else echo $PWD/variants/$1/libripplemq_engine.so; fi; }
for rep in 1 2; do
  for v in cur t512; do
    RMQ_LIB=$(lib $v) timeout -k 10 200 python bench.py --steps 200 --warmup 20 $Q > gpurun_out/${T}_${v}_B_$rep.json 2>&1 || exit 1
  done
done
for v in cur t512; do
  RMQ_LIB=$(lib $v) timeout -k 10 200 python bench.py --config D --pool 16 --steps 40 --warmup 5 $Q > gpurun_out/${T}_${v}_D_1.json 2>&1 || exit 1
done
