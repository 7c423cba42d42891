# A/B of 512-record ranking tiles (variants/tile9, built with -DRMQ_TILE_BITS=9) against
# the default 1024-record tiles: the GPU parity suite on the variant, then the driver-shaped line
# (--steps 20, 3 pairs) and a steady line (400 steps, 2 pairs), and config D (1 pair).
# usage: bash tools/gpu_tile9.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1
mkdir -p gpurun_out
V=$PWD/variants/tile9/libripplemq_engine.so
C=$PWD/ripplemq_amd/libripplemq_engine.so
RMQ_LIB=$V timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "not config_A and not 20000 and not full" > gpurun_out/${T}_pytest_tile9.txt 2>&1 || echo "variant parity failed (see log)"
Q="--no-cpu-baseline --fetch-rounds 0 --host-steps 0"
for rep in 1 2 3; do
  for v in cur tile9; do
    if [ $v = cur ]; then L=$C; else L=$V; fi
    RMQ_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 $Q > gpurun_out/${T}_${v}_20_$rep.json 2>&1 || exit 1
  done
done
for rep in 1 2; do
  for v in cur tile9; do
    if [ $v = cur ]; then L=$C; else L=$V; fi
    RMQ_LIB=$L timeout -k 10 200 python bench.py --steps 400 --warmup 40 $Q > gpurun_out/${T}_${v}_400_$rep.json 2>&1 || exit 1
  done
done
for v in cur tile9; do
  if [ $v = cur ]; then L=$C; else L=$V; fi
  RMQ_LIB=$L timeout -k 10 200 python bench.py --config D --pool 16 --steps 100 --warmup 10 $Q > gpurun_out/${T}_${v}_D.json 2>&1 || exit 1
done
