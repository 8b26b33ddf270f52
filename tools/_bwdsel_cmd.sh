#!/bin/bash
# GPU box: backward with the selector words read through L1 instead of staged in LDS
# (bwd_sel_lds=2), which widens the column blocks where the block count allows (k = 8).
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bwd_opts_sweep.py --k 8 --opts '[{}, {"bwd_sel_lds": 2}, {"bwd_sel_lds": 2, "bwd_unroll": 8}, {"bwd_sel_lds": 2, "bwd_features_per_lane": 4}, {"bwd_features_per_lane": 4}, {}]' > gpurun_out/bwdsel.jsonl 2> gpurun_out/bwdsel.err || exit $?
timeout -k 10 300 python -u tools/bwd_opts_sweep.py --k 16 --opts '[{}, {"bwd_sel_lds": 2}]' >> gpurun_out/bwdsel.jsonl 2>> gpurun_out/bwdsel.err || exit $?
cat gpurun_out/bwdsel.jsonl
