# Dispatch order of the pipeline roles: stage 3 last (default) vs first (RMQ_S3_FIRST=1).
set -e
R=$GRAFT_REPO_ROOT
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for o in 0 1; do for g in 2 4; do
RMQ_S3_FIRST=$o timeout -k 10 200 python bench.py --group $g --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/ord_${o}_g$g.json 2> gpurun_out/ord_${o}_g$g.err
done; done
RMQ_S3_FIRST=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_s3f.log 2>&1
