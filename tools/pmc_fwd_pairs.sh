#!/bin/bash
# PMC of the Reddit k=16 forward with pair-chunk records (the round-6 default)
# against the packed records it replaced (fwd_chunk3=2), same passes as tools/pmc_fwd_layout.sh
# plus the L2-to-fabric read requests split by DRAM (tooling). Summarise with
#   python tools/pmc_summary.py gpurun_out/pmc_fp_pairs ; ... gpurun_out/pmc_fp_records
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export PMC_K=16
PASSES="SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS
SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS
TD_TD_BUSY_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"
for v in pairs:'{}' records:'{"fwd_chunk3": 2}'; do
  tag=${v%%:*}; opts=${v#*:}
  PMC_TAG="_fp_$tag" PMC_OPTS="$opts" PMC_PASSES="$PASSES" bash "$ROOT/tools/pmc_run.sh" || exit $?
done
