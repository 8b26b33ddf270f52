set -e
P="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY
TD_TD_BUSY_sum GRBM_GUI_ACTIVE TA_TA_BUSY_sum"
for w in 4 8; do
  for k in 16 32; do
    PMC_K=$k PMC_OPTS="{\"fwd_waves\": $w, \"fwd_handout\": 2}" PMC_TAG="_w${w}_k${k}" PMC_PASSES="$P" bash tools/pmc_run.sh
  done
done
