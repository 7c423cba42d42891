# A/B of the eager first launch on an idle pipeline (RMQ_EAGER_START=1, default) against waiting for
# a full group (=0), same library: GPU parity suite, then the driver-shaped line (4 pairs) and the
# steady line (1 pair). usage: bash tools/gpu_eager.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || exit 1
Q="--no-cpu-baseline --fetch-rounds 0 --host-steps 0"
for rep in 1 2 3 4; do
  for v in 1 0; do
    RMQ_TRACE=1 RMQ_EAGER_START=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 $Q > gpurun_out/${T}_e${v}_20_$rep.json 2> gpurun_out/${T}_e${v}_20_$rep.err || exit 1
  done
done
for v in 1 0; do
  RMQ_EAGER_START=$v timeout -k 10 200 python bench.py --steps 400 --warmup 40 $Q > gpurun_out/${T}_e${v}_400_1.json 2>&1 || exit 1
done
