# Kernel traces of the pipeline in three launch shapes (diagnostic): fused (RMQ_SPLIT=0), split
# side by side (default), split one after the other (RMQ_SPLIT=2). Run through gpurun.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
T=${1:-r05f}
Q="--no-cpu-baseline --fetch-rounds 0 --concurrent-rounds 0 --host-steps 0 --tier-rounds 0"
for sp in 0 1 2; do
  (cd /tmp && export TMPDIR=/tmp && RMQ_SPLIT=$sp timeout -s KILL 120 rocprofv3 --kernel-trace -f csv -d "$R/gpurun_out/${T}_kt$sp" -o kt -- python3 "$R/bench.py" --steps 60 --warmup 10 $Q) > "$R/gpurun_out/${T}_kt$sp.log" 2>&1 || { tail -20 "$R/gpurun_out/${T}_kt$sp.log"; exit 1; }
done
