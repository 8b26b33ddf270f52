#!/bin/bash
# rocprofv3 PMC passes over tools/pmc_driver.py (one counter group per pass, --kernel-trace
# only beside --pmc). Output: gpurun_out/pmc/<pass>/... ; summarise with tools/pmc_summary.py
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmc${PMC_TAG}"
mkdir -p "$OUT"
export PMC_OUT="$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i + 1))
  timeout -k 10 240 rocprofv3 --pmc $counters --kernel-trace --output-format csv \
    -d "$OUT/pass$i" -o run -- python3 "$ROOT/tools/pmc_driver.py" > "$OUT/pass$i.log" 2>&1
  rc=$?
  echo "pass $i ($counters): rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done <<LIST
${PMC_PASSES:-FETCH_SIZE
WRITE_SIZE
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_READ_sum
SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum}
LIST
