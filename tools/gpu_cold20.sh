# First-launch cost of the driver-shaped bench: kernel traces of --steps 20 with the default pool
# (every timed batch touched for the first time), a pool of 8 (batches reused), and warmup over the
# whole pool. usage: bash tools/gpu_cold20.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
run() {
  n=$1; shift
  timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/${T}_${n}_kt -o kt -- python3 $R/bench.py --steps 20 --no-cpu-baseline --fetch-rounds 0 --host-steps 0 "$@" > $R/gpurun_out/${T}_${n}.json 2>&1 || exit 1
  python3 $R/tools/trace_launches.py $R/gpurun_out/${T}_${n}_kt/kt_kernel_trace.csv > $R/gpurun_out/${T}_${n}_launches.txt
}
run w5 --warmup 5
run p8 --warmup 5 --pool 8
run w48 --warmup 48
