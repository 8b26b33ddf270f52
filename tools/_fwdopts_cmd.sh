cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -5 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for k in 16 32 64; do
timeout -k 10 300 python -u tools/fwd_opts_sweep.py --k $k --opts '[{}, {"fwd_rot_windows": 16, "fwd_rot_rate": 160, "quad_loads": 2}]' >> gpurun_out/fwdopts3.jsonl 2>> gpurun_out/fwdopts.err || exit $?
done
timeout -k 10 300 python -u tools/fwd_fixed_sweep.py --k 8,16,32,64 --dataset ogbn-proteins >> gpurun_out/fwdopts3.jsonl 2>> gpurun_out/fwdopts.err || exit $?
cat gpurun_out/fwdopts3.jsonl
