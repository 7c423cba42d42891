# Launch-group sizes 4 / 6 / 8 with the 16-lane stage 2.
set -e
R=$GRAFT_REPO_ROOT
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for g in 4 6 8; do
timeout -k 10 200 python bench.py --group $g --steps 1200 --warmup 120 --no-cpu-baseline > gpurun_out/g2_g$g.json 2> gpurun_out/g2_g$g.err
done
RMQ_STAMPS_AT=15 RMQ_STAMPS=gpurun_out/st2_g8.csv timeout -k 10 240 python bench.py --group 8 --steps 200 --warmup 50 --no-cpu-baseline > gpurun_out/bs2_g8.log 2>&1
