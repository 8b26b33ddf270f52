#!/bin/bash
# Counters behind the backward bound model and the two-pass byte budget
# (tooling): for each dataset:kind:k of PMC_CONFIGS, four rocprofv3 --pmc passes over
# tools/pmc_driver.py (instruction mix + LDS; texture path + L1 misses; L2 hits and fabric
# requests; writes), each its own run with --kernel-trace only. Output gpurun_out/pmc_model_<tag>/;
# summarise with  python tools/pmc_group.py gpurun_out/pmc_model_<tag>
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
CONFIGS="${PMC_CONFIGS:-reddit:sage:16 reddit:sage:32 reddit:sage:64 ogbn-products:sage:32}"
for c in $CONFIGS; do
  IFS=: read -r ds kind k <<< "$c"
  export PMC_DATASET=$ds PMC_KIND=$kind PMC_K=$k PMC_TAG="_model_${ds}_k${k}"
  PMC_PASSES="SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS
TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum
TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" bash "$ROOT/tools/pmc_run.sh" || exit $?
done
