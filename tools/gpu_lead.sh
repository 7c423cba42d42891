# Stage-3 lead sweep (RMQ_S3_LEAD = stage-3 workgroups dispatched before ranking and scans): GPU
# parity tests of the pipeline, then the steady line (500 steps) and the 20-step line per setting,
# and phase stamps at the best candidate. usage: bash tools/gpu_lead.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1
mkdir -p gpurun_out
RMQ_S3_LEAD=1536 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.txt 2>&1 || exit 1
Q="--no-cpu-baseline --fetch-rounds 0 --host-steps 0"
for rep in 1 2; do
  for L in 0 1024 1280 1536 1792; do
    RMQ_S3_LEAD=$L timeout -k 10 200 python bench.py --steps 500 --warmup 50 $Q > gpurun_out/${T}_L${L}_500_$rep.json 2>&1 || exit 1
  done
done
for L in 0 1280 1536; do
  RMQ_S3_LEAD=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 $Q > gpurun_out/${T}_L${L}_20.json 2>&1 || exit 1
done
RMQ_S3_LEAD=1536 RMQ_STAMPS=gpurun_out/${T}_st.csv RMQ_STAMPS_AT=100 timeout -k 10 200 python bench.py --steps 300 --warmup 30 $Q > gpurun_out/${T}_stamped.json 2>&1 || exit 1
python tools/pipe_stamps.py gpurun_out/${T}_st.csv > gpurun_out/${T}_stamps.txt 2>&1
