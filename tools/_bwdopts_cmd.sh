cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bwd_opts_sweep.py --k 64 --opts '[{}, {"bwd_slot_groups": 4}, {"bwd_slot_groups": 4, "bwd_waves": 8}, {"bwd_slot_groups": 2, "bwd_waves": 16}, {"bwd_slot_groups": 2, "bwd_unroll": 12}, {"bwd_slot_groups": 2, "bwd_tasks_per_cu": 1}, {"bwd_slot_groups": 8}]' > gpurun_out/bwdk.jsonl 2> gpurun_out/bwdk.err || exit $?
timeout -k 10 300 python -u tools/bwd_opts_sweep.py --k 32 --opts '[{}, {"bwd_slot_groups": 4}, {"bwd_slot_groups": 2, "bwd_waves": 8}, {"bwd_slot_groups": 2, "bwd_waves": 16}, {"bwd_slot_groups": 2, "bwd_unroll": 12}, {"bwd_slot_groups": 2, "bwd_features_per_lane": 2}]' >> gpurun_out/bwdk.jsonl 2>> gpurun_out/bwdk.err || exit $?
cat gpurun_out/bwdk.jsonl
