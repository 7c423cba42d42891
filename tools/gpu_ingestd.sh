# GPU parity suite, then config D over the in-process transport (2 ranks on one GPU: follower
# ingest of large records) for the current library and variants/head, and the migrate kernel time.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
T=$1
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || exit 1
for v in cur head; do
  if [ $v = cur ]; then L=$PWD/ripplemq_amd/libripplemq_engine.so; else L=$PWD/variants/head/libripplemq_engine.so; fi
  RMQ_LIB=$L timeout -k 10 300 python bench.py --gpus 2 --transport local --config D --pool 8 --steps 40 --warmup 5 --no-cpu-baseline --fetch-rounds 0 --host-steps 0 > gpurun_out/${T}_${v}_localD.json 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${T}_prof -o kt -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --fetch-rounds 0 --host-steps 0 > $R/gpurun_out/${T}_prof.log 2>&1
