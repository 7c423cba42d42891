# Three-way A/B: the current library (cur), variants/head (the last commit) and variants/tile9 (the
# last commit with 512-record tiles): GPU parity suite on cur, then the driver-shaped line
# (3 rounds) and the steady line (2 rounds), rotating the libraries inside each round.
# usage: bash tools/gpu_ab3.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || exit 1
Q="--no-cpu-baseline --fetch-rounds 0 --host-steps 0"
lib() { if [ $1 = cur ]; then echo $PWD/ripplemq_amd/libripplemq_engine.so; else echo $PWD/variants/$1/libripplemq_engine.so; fi; }
for rep in 1 2 3; do
  for v in cur head tile9; do
    RMQ_LIB=$(lib $v) timeout -k 10 200 python bench.py --steps 20 --warmup 5 $Q > gpurun_out/${T}_${v}_20_$rep.json 2>&1 || exit 1
  done
done
for rep in 1 2; do
  for v in cur head tile9; do
    RMQ_LIB=$(lib $v) timeout -k 10 200 python bench.py --steps 400 --warmup 40 $Q > gpurun_out/${T}_${v}_400_$rep.json 2>&1 || exit 1
  done
done
