# Occupancy: default build (4 waves per SIMD, no spills) vs 6 waves per SIMD (3 workgroups per CU,
# VGPR spills). Variant build: make -C ripplemq_amd/csrc BUILD=../../build/w6
# OUT=../../variants/libw6.so CXXFLAGS="... -DRMQ_PIPE_WAVES_PER_SIMD=6"
set -e
R=$GRAFT_REPO_ROOT
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/occ_4.json 2> gpurun_out/occ_4.err
RMQ_LIB=$R/variants/libw6.so timeout -k 10 200 python bench.py --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/occ_6.json 2> gpurun_out/occ_6.err
