set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && echo TESTS_OK &&
timeout -k 10 300 python -u tools/configs_time.py --out gpurun_out/configs.json > gpurun_out/configs.log 2>&1 && echo CONFIGS_OK &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 && echo BENCH_OK
