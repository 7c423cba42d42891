# Kernel stats of the 2-rank rehearsal for the current library and variants/<V>. bash tools/kt_local2.sh <tag> <V>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
T=$1; V=$2
Q="--gpus 2 --transport local --steps 100 --warmup 10 --segment-mb 2 --pool 8 --no-cpu-baseline --fetch-rounds 0 --concurrent-rounds 0 --host-steps 0 --tier-rounds 0"
for v in cur $V; do
  if [ $v = cur ]; then L=$R/ripplemq_amd/libripplemq_engine.so; else L=$R/variants/$V/libripplemq_engine.so; fi
  (cd /tmp && export TMPDIR=/tmp && RMQ_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/${T}_kt_$v" -o kt -- python3 "$R/bench.py" $Q) > "$R/gpurun_out/${T}_kt_$v.log" 2>&1 || exit 1
  echo "== $v"; cut -d, -f1-4 gpurun_out/${T}_kt_$v/kt_kernel_stats.csv | grep -i "ingest\|pipeline"
done
