# Ring-pool round: new parity tests, then bench lines with load-sized and equal rings, and config D.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "config_d_shape or rejected_long or set_segments" > gpurun_out/rings_pytest.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/rings_b_load.json 2> gpurun_out/rings_b_load.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --fetch-rounds 0 > gpurun_out/rings_b_load20.json 2>> gpurun_out/rings_b_load.err &&
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --rings equal --fetch-rounds 0 > gpurun_out/rings_b_equal.json 2> gpurun_out/rings_b_equal.err &&
timeout -k 10 300 python bench.py --config D --steps 100 --warmup 10 --no-cpu-baseline --pool 16 > gpurun_out/rings_d.json 2> gpurun_out/rings_d.err
