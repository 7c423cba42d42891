# Round-2 check of the 256-thread pipeline default: GPU parity suite, A/B against the 512-thread
# library (variants/t512) on the driver-shaped line (3 pairs), the steady line (2 pairs) and config D,
# then the default bench line (fetch leg included) and rocprofv3 kernel stats of it.
# usage: bash tools/gpu_r02b.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
T=$1
mkdir -p gpurun_out
V=$PWD/variants/t512/libripplemq_engine.so
C=$PWD/ripplemq_amd/libripplemq_engine.so
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.txt 2>&1 || exit 1
Q="--no-cpu-baseline --fetch-rounds 0 --host-steps 0"
for rep in 1 2 3; do
  for v in cur t512; do
    if [ $v = cur ]; then L=$C; else L=$V; fi
    RMQ_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 $Q > gpurun_out/${T}_${v}_20_$rep.json 2>&1 || exit 1
  done
done
for rep in 1 2; do
  for v in cur t512; do
    if [ $v = cur ]; then L=$C; else L=$V; fi
    RMQ_LIB=$L timeout -k 10 200 python bench.py --steps 400 --warmup 40 $Q > gpurun_out/${T}_${v}_400_$rep.json 2>&1 || exit 1
  done
done
for v in cur t512; do
  if [ $v = cur ]; then L=$C; else L=$V; fi
  RMQ_LIB=$L timeout -k 10 200 python bench.py --config D --pool 16 --steps 100 --warmup 10 $Q > gpurun_out/${T}_${v}_D.json 2>&1 || exit 1
done
timeout -k 10 300 python bench.py --no-cpu-baseline --host-steps 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${T}_kt -o kt -- python3 $R/bench.py --steps 400 --warmup 40 --no-cpu-baseline --host-steps 0 > $R/gpurun_out/${T}_kt.log 2>&1 || exit 1
