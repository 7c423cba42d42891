# A/B of the current library against variants/head on configs B and D (bench lines), after the
# GPU parity suite. usage: bash tools/gpu_abd.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || exit 1
for rep in 1 2; do
  for v in cur head; do
    if [ $v = cur ]; then L=$PWD/ripplemq_amd/libripplemq_engine.so; else L=$PWD/variants/head/libripplemq_engine.so; fi
    RMQ_LIB=$L timeout -k 10 200 python bench.py --steps 400 --warmup 40 --no-cpu-baseline --fetch-rounds 0 --host-steps 0 > gpurun_out/${T}_${v}_B_$rep.json 2>&1 || exit 1
    RMQ_LIB=$L timeout -k 10 200 python bench.py --config D --pool 16 --steps 100 --warmup 10 --no-cpu-baseline --fetch-rounds 0 --host-steps 0 > gpurun_out/${T}_${v}_D_$rep.json 2>&1 || exit 1
  done
done
