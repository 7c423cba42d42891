# A/B of the current library against variants/head on the driver-shaped line (--steps 20
# --warmup 5, 4 pairs) and the steady line (400 steps, 1 pair), after the GPU parity suite.
# usage: bash tools/gpu_ab20.sh <tag> [skip-tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1
mkdir -p gpurun_out
if [ -z "$2" ]; then
  timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || exit 1
fi
Q="--no-cpu-baseline --fetch-rounds 0 --host-steps 0"
for rep in 1 2 3 4; do
  for v in cur head; do
    if [ $v = cur ]; then L=$PWD/ripplemq_amd/libripplemq_engine.so; else L=$PWD/variants/head/libripplemq_engine.so; fi
    RMQ_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 $Q > gpurun_out/${T}_${v}_20_$rep.json 2>&1 || exit 1
  done
done
for v in cur head; do
  if [ $v = cur ]; then L=$PWD/ripplemq_amd/libripplemq_engine.so; else L=$PWD/variants/head/libripplemq_engine.so; fi
  RMQ_LIB=$L timeout -k 10 200 python bench.py --steps 400 --warmup 40 $Q > gpurun_out/${T}_${v}_400_1.json 2>&1 || exit 1
done
