set -o pipefail
mkdir -p gpurun_out
for k in 0 3 7 15; do
  echo "RMQ_COPY_THREADS=$k" >> gpurun_out/hostprobe.txt
  RMQ_COPY_THREADS=$k timeout -k 10 120 python tools/host_probe.py >> gpurun_out/hostprobe.txt 2>&1 || exit 1
done
