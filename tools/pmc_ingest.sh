# Counters of the follower ingest kernels in the 2-rank rehearsal (diagnostic). Run through gpurun:
#   bash tools/pmc_ingest.sh <tag> [sq|mem]; then KSUB=ingest_verify python3 tools/pmc_show.py gpurun_out/<tag>_pmc*
set -o pipefail
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
T=${1:-r05i}
WHAT=${2:-sq}
Q="--gpus 2 --transport local --steps 100 --warmup 10 --segment-mb 2 --pool 8 --no-cpu-baseline --fetch-rounds 0 --concurrent-rounds 0 --host-steps 0 --tier-rounds 0"
if [ "$WHAT" = sq ]; then
  SETS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
        "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR")
else
  SETS=("TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum"
        "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE")
fi
k=0
for set in "${SETS[@]}"; do
  k=$((k+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $set -f csv -d "$R/gpurun_out/${T}_pmc$k" -o pm -- python3 "$R/bench.py" $Q) > "$R/gpurun_out/${T}_pmc$k.log" 2>&1 || { echo "pass $k failed"; tail -5 "$R/gpurun_out/${T}_pmc$k.log"; exit 1; }
done
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/${T}_kt" -o kt -- python3 "$R/bench.py" $Q) > "$R/gpurun_out/${T}_kt.log" 2>&1 || exit 1
