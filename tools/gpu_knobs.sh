# Timing knobs at the default launch group (RMQ_DEBUG bits, results invalid when set): what each
# part of the launch costs. 1 no payload ring stores, 2 no CRC lookups, 4 no payload loads,
# 8 no CRC tables, 16 skip stages 1-2.
set -e
R=$GRAFT_REPO_ROOT
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for d in ${FLAGS:-0 1 2 4 8 10 16 27}; do
RMQ_DEBUG=$d timeout -k 10 200 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/knob_$d.json 2> gpurun_out/knob_$d.err
done
