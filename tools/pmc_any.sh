#!/bin/bash
# rocprofv3 PMC passes over an arbitrary python command (tooling): one counter group per pass,
# --kernel-trace only beside --pmc. Usage: PMC_TAG=x tools/pmc_any.sh script.py [args]
# Output gpurun_out/pmcany_<tag>/pass<i>/; summarise with tools/pmc_group.py <dir>
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmcany_${PMC_TAG:-x}"
mkdir -p "$OUT"
SCRIPT="$ROOT/$1"; shift
cd /tmp && export TMPDIR=/tmp
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i + 1))
  timeout -k 10 240 rocprofv3 --pmc $counters --kernel-trace --output-format csv \
    -d "$OUT/pass$i" -o run -- python3 "$SCRIPT" "$@" > "$OUT/pass$i.log" 2>&1
  rc=$?
  echo "pass $i ($counters): rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done <<LIST
${PMC_PASSES:-TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_READ_sum
SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE}
LIST
