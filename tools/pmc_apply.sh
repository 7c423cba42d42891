# SQ counters of the split pipeline's launches (diagnostic; RMQ_SPLIT=2: apply and rank launches
# one after the other, so each dispatch is one role set). Run through gpurun.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
T=${1:-r05g}
Q="--no-cpu-baseline --fetch-rounds 0 --concurrent-rounds 0 --host-steps 0 --tier-rounds 0"
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 30 rocprofv3 -L) > "$R/gpurun_out/${T}_avail.txt" 2>&1 || true
k=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR"; do
  k=$((k+1))
  (cd /tmp && export TMPDIR=/tmp && RMQ_SPLIT=2 timeout -s KILL 90 rocprofv3 --pmc $set -f csv -d "$R/gpurun_out/${T}_pmc$k" -o pm -- python3 "$R/bench.py" --steps 60 --warmup 10 $Q) > "$R/gpurun_out/${T}_pmc$k.log" 2>&1 || { echo "pass $k failed"; tail -5 "$R/gpurun_out/${T}_pmc$k.log"; }
done
