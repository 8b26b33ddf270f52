#!/bin/bash
# GPU box: forward CBSR record stride re-check on the fixed-point kernel (80/96-B records:
# a smaller, more L2-resident table at the cost of records that straddle two lines).
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/fwd_opts_sweep.py --k 16 --opts '[{}, {"fwd_record_bytes": 80}, {"fwd_record_bytes": 96}, {"fwd_record_bytes": 80, "fwd_rot_rate": 330}, {}]' > gpurun_out/fwdrec.jsonl 2> gpurun_out/fwdrec.err || exit $?
timeout -k 10 300 python -u tools/fwd_opts_sweep.py --k 8 --opts '[{}, {"fwd_chunk3": 2, "fwd_record_bytes": 48}, {"fwd_chunk3": 2, "fwd_record_bytes": 64}, {}]' >> gpurun_out/fwdrec.jsonl 2>> gpurun_out/fwdrec.err || exit $?
timeout -k 10 300 python -u tools/fwd_opts_sweep.py --k 32 --opts '[{}, {"fwd_two_tables": 2, "fwd_record_bytes": 160}, {"fwd_two_tables": 2, "fwd_record_bytes": 256}, {}]' >> gpurun_out/fwdrec.jsonl 2>> gpurun_out/fwdrec.err || exit $?
cat gpurun_out/fwdrec.jsonl
