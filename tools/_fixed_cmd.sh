cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/fwd_fixed_sweep.py > gpurun_out/fixed_sweep.jsonl 2> gpurun_out/fixed_sweep.err || exit $?
timeout -k 10 300 python -u tools/fwd_fixed_sweep.py --k 8,16 --opts '{"fwd_chunk3": 2}' >> gpurun_out/fixed_sweep.jsonl 2>> gpurun_out/fixed_sweep.err || exit $?
timeout -k 10 300 python -u tools/fwd_fixed_sweep.py --k 8,16,32,64 --dataset ogbn-proteins >> gpurun_out/fixed_sweep.jsonl 2>> gpurun_out/fixed_sweep.err || exit $?
timeout -k 10 300 python -u tools/fwd_fixed_sweep.py --k 16,32 --dataset ogbn-products >> gpurun_out/fixed_sweep.jsonl 2>> gpurun_out/fixed_sweep.err || exit $?
cat gpurun_out/fixed_sweep.jsonl
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_fixed -o fx --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/fwd_fixed_sweep.py --k 16 > /dev/null 2>&1) || exit $?
