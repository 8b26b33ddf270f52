#!/bin/bash
# PMC of the locality cases: the community graph shuffled with the identity and
# the clustered column order (backward L1-miss requests, L2 hit), and in ID order / shuffled at
# k = 64 (forward L2 hit). Three passes each (tools/pmc_run.sh), output
# gpurun_out/pmc_loc_<graph>_<order>_k<k>/; summarise with
#   python tools/pmc_traffic.py --locality gpurun_out
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
CASES="${PMC_LOC_CASES:-shuffled:identity:16 shuffled:clustered:16 community:identity:64 shuffled:identity:64 shuffled:clustered:64}"
for c in $CASES; do
  IFS=: read -r graph order k <<< "$c"
  case $order in
    identity) opts='{}' ;;
    clustered) opts='{"col_order": 3}' ;;
    *) echo "unknown order $order"; exit 2 ;;
  esac
  export PMC_GRAPH=$graph PMC_OPTS="$opts" PMC_K=$k PMC_TAG="_loc_${graph}_${order}_k${k}"
  PMC_PASSES="FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" bash "$ROOT/tools/pmc_run.sh" || exit $?
done
