# Stage-2 lanes per partition column: default build (16), 16, 32 (variant builds via RMQ_LIB).
# Variant builds: make -C ripplemq_amd/csrc BUILD=../../build/vN OUT=../../variants/libN.so CXXFLAGS="... -DRMQ_SCAN_LANES=N"
set -e
R=$GRAFT_REPO_ROOT
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for v in 8 16 32; do
L=""; [ $v != 8 ] && L=$R/variants/lib$v.so
RMQ_LIB=$L timeout -k 10 200 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/sl_$v.json 2> gpurun_out/sl_$v.err
RMQ_LIB=$L RMQ_STAMPS_AT=30 RMQ_STAMPS=gpurun_out/st_sl$v.csv timeout -k 10 240 python bench.py --steps 200 --warmup 50 --no-cpu-baseline > gpurun_out/bs_sl$v.log 2>&1
done
