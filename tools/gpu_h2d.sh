set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 python tools/h2d_probe.py > gpurun_out/h2d.txt 2>&1 &&
echo "HSA_ENABLE_SDMA=0" >> gpurun_out/h2d.txt &&
HSA_ENABLE_SDMA=0 timeout -k 10 180 python tools/h2d_probe.py >> gpurun_out/h2d.txt 2>&1
