# Host-path round: GPU parity suite, then the default bench line (device leg, host leg, fetch leg).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/host_pytest.txt 2>&1 &&
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/host_bench.json 2> gpurun_out/host_bench.err
