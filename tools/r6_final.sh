#!/bin/bash
# Round-6 measurement set on the final library (tooling): PMC traffic of every BASELINE
# config (profiles/pmc_traffic.json), the N=1 bench line, its rocprofv3 kernel statistics,
# the N=2 gloo rehearsal through the bare command, every rank of an 8-GPU shard, the configs,
# the Reddit k=16 autograd step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
bash tools/gpu_job.sh \
  'r6f_pmc|900|bash tools/pmc_configs.sh' \
  'r6f_ptraf|120|python tools/pmc_traffic.py --all gpurun_out --out gpurun_out/pmc_traffic.json' \
  'r6f_bench|400|python3 bench.py --gpus 1 --steps 20 --warmup 5 --traffic-json gpurun_out/pmc_traffic.json' \
  'r6f_bprof|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r6f_bprof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-comparator --k-sweep "" --traffic-json $GRAFT_REPO_ROOT/gpurun_out/pmc_traffic.json' \
  'r6f_w2|300|MAXK_BENCH_BACKEND=gloo python3 bench.py --gpus 2 --steps 10 --warmup 3' \
  'r6f_shard8|300|python -u tools/shard_time.py --worlds 8 --all-ranks --layouts records' \
  'r6f_configs|600|python -u tools/configs_time.py --out gpurun_out/r6f_configs.json' \
  'r6f_auto|300|python -u tools/autograd_step.py'
