# Stage-1 tile of 1024 (default build) vs 2048 records (variant build via RMQ_LIB), then the
# parity tests on the 2048 build.
# Variant build: make -C ripplemq_amd/csrc BUILD=../../build/t11 OUT=../../variants/libt11.so CXXFLAGS="... -DRMQ_TILE_BITS=11"
set -e
R=$GRAFT_REPO_ROOT
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for v in 10 11; do
L=""; [ $v != 10 ] && L=$R/variants/libt$v.so
for g in 2 4; do
RMQ_LIB=$L timeout -k 10 200 python bench.py --group $g --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/tile_${v}_g$g.json 2> gpurun_out/tile_${v}_g$g.err
done; done
RMQ_LIB=$R/variants/libt11.so RMQ_STAMPS_AT=30 RMQ_STAMPS=gpurun_out/st_t11.csv timeout -k 10 240 python bench.py --steps 200 --warmup 50 --no-cpu-baseline > gpurun_out/bs_t11.log 2>&1
RMQ_LIB=$R/variants/libt11.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_t11.log 2>&1
