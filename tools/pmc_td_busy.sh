#!/bin/bash
# Texture-path busy fraction of the current kernels (tooling, round 5): one PMC pass of
# TD/TA busy and GRBM_GUI_ACTIVE over tools/pmc_driver.py at each k (Reddit, defaults).
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for k in 16 64; do
  PMC_K=$k PMC_TAG="_td_k$k" PMC_PASSES="TD_TD_BUSY_sum GRBM_GUI_ACTIVE TA_TA_BUSY_sum
TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY" \
    bash "$ROOT/tools/pmc_run.sh" || exit $?
done
