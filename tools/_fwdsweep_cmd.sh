#!/bin/bash
# GPU box: forward option re-check after the fixed-point retune (tile rows, waves, unroll,
# two tables, prefetch) at k = 16 / 32 / 8 on the Reddit-shaped graph.
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/fwd_opts_sweep.py --k 16 --opts '[{}, {"fwd_two_tables": 1}, {"fwd_tile_rows": 64}, {"fwd_tile_rows": 16}, {"fwd_waves": 8}, {"fwd_waves": 6}, {"fwd_unroll": 16}, {"fwd_prefetch": 1}, {}]' > gpurun_out/fwdk.jsonl 2> gpurun_out/fwdk.err || exit $?
timeout -k 10 300 python -u tools/fwd_opts_sweep.py --k 32 --opts '[{}, {"fwd_two_tables": 2}, {"fwd_tile_rows": 64}, {"fwd_waves": 8}, {"fwd_unroll": 16}, {}]' >> gpurun_out/fwdk.jsonl 2>> gpurun_out/fwdk.err || exit $?
timeout -k 10 300 python -u tools/fwd_opts_sweep.py --k 8 --opts '[{}, {"fwd_fixed": 1}, {"fwd_tile_rows": 64}, {"fwd_waves": 8}, {"fwd_unroll": 16}, {}]' >> gpurun_out/fwdk.jsonl 2>> gpurun_out/fwdk.err || exit $?
cat gpurun_out/fwdk.jsonl
