# Counters of the split pipeline's launches (diagnostic; RMQ_SPLIT=2: apply and rank launches one
# after the other, so each dispatch is one role set; SPLIT=0 keeps the one launch, e.g. with
# RMQ_S3_ROLES; CFG=D: config D). Run through gpurun:
#   bash tools/pmc_apply.sh <tag> [sq|mem]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; R=$GRAFT_REPO_ROOT
T=${1:-r05g}
WHAT=${2:-sq}
Q="${CFG:+--config $CFG --pool 16} --no-cpu-baseline --fetch-rounds 0 --concurrent-rounds 0 --host-steps 0 --tier-rounds 0"
if [ "$WHAT" = sq ]; then
  SETS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
        "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR")
else
  SETS=("TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_SERIALIZATION_STALL_sum GRBM_GUI_ACTIVE"
        "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum"
        "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum")
fi
k=0
for set in "${SETS[@]}"; do
  k=$((k+1))
  (cd /tmp && export TMPDIR=/tmp && RMQ_SPLIT=${SPLIT:-2} timeout -s KILL 90 rocprofv3 --pmc $set -f csv -d "$R/gpurun_out/${T}_pmc$k" -o pm -- python3 "$R/bench.py" --steps 60 --warmup 10 $Q) > "$R/gpurun_out/${T}_pmc$k.log" 2>&1 || { echo "pass $k failed"; tail -5 "$R/gpurun_out/${T}_pmc$k.log"; }
done
