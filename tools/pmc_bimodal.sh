#!/bin/bash
# PMC passes over tools/shard_bimodal.py (tooling, round 5): which counters separate the fast
# and the slow plan instances of an 8-GPU rank's backward. Each pass carries its
# own kernel trace, so instances are classified by duration within the pass; summarise with
#   python tools/pmc_bimodal_summary.py gpurun_out/pmc_bimodal
PMC_PASSES="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY
TD_TD_BUSY_sum GRBM_GUI_ACTIVE TA_TA_BUSY_sum
TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum TCC_TAG_STALL_sum"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmc_bimodal"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i + 1))
  timeout -k 10 240 rocprofv3 --pmc $counters --kernel-trace --output-format csv \
    -d "$OUT/pass$i" -o run -- python3 "$ROOT/tools/shard_bimodal.py" --rank 3 --plans 8 \
    > "$OUT/pass$i.log" 2>&1
  rc=$?
  echo "pass $i ($counters): rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done <<LIST
$PMC_PASSES
LIST
