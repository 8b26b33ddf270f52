#!/bin/bash
# Texture-path / L1 / L2 / SQ counters of the SSpMM backward (and the forward) under a few plan
# option sets, one rocprofv3 pass per counter group (tools/pmc_run.sh), Reddit-shaped graph,
# k = PMC_K (16). Output gpurun_out/pmc_cmp_<i>/; summarise with
#   python tools/pmc_summary.py gpurun_out/pmc_cmp_<i>
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
i=0
for opts in "$@"; do
  export PMC_OPTS="$opts" PMC_TAG="_cmp_$i"
  echo "== set $i: $opts"
  PMC_PASSES="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE
TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TOTAL_READ_sum
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
TCC_HIT_sum TCC_MISS_sum" bash "$ROOT/tools/pmc_run.sh" || exit $?
  i=$((i + 1))
done
