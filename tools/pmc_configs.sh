#!/bin/bash
# PMC traffic of the BASELINE configs (config 4's "rocprof HBM GB/s" and the k sweep):
# for each dataset:kind:k, three rocprofv3 passes over tools/pmc_driver.py (FETCH_SIZE;
# WRITE_SIZE; TCC hit/miss + L1-miss requests), each its own run with --kernel-trace only
# (counter limits: MI355X_MICROARCH.md "rocprofv3 PMC slots"). Output gpurun_out/pmc_<tag>/;
# summarise with  python tools/pmc_traffic.py --all gpurun_out
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
CONFIGS="${PMC_CONFIGS:-reddit:sage:8 reddit:sage:16 reddit:sage:32 reddit:sage:64 ogbn-products:sage:32 ogbn-proteins:gcn:8 ogbn-proteins:gcn:16 ogbn-proteins:gcn:32 ogbn-proteins:gcn:64}"
for c in $CONFIGS; do
  IFS=: read -r ds kind k <<< "$c"
  export PMC_DATASET=$ds PMC_KIND=$kind PMC_K=$k PMC_TAG="_${ds}_${kind}_k${k}"
  PMC_PASSES="FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" bash "$ROOT/tools/pmc_run.sh" || exit $?
done
