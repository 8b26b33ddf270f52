#!/bin/bash
# PMC passes over tools/shard_alloc.py --plans-only (tooling, round 6): address-translation,
# texture-path and L2 counters of an 8-GPU rank's backward on the shard's plan and eight fresh
# plans. Each pass is its own process (its own plan placements) with its own
# kernel trace, so plans are classified fast / slow by duration within the pass. Summarise:
#   python tools/pmc_alloc_summary.py gpurun_out/pmc_alloc
PMC_PASSES="${PMC_PASSES:-TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_PERMISSION_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE
TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum
TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_TAG_STALL_sum}"
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmc_alloc${PMC_TAG}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $counters --kernel-trace --output-format csv \
    -d "$OUT/pass$i" -o run -- python3 "$ROOT/tools/shard_alloc.py" --plans-only --plans 8 \
    --reps 10 > "$OUT/pass$i.log" 2>&1
  rc=$?
  echo "pass $i ($counters): rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done <<LIST
$PMC_PASSES
LIST
