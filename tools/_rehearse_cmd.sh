#!/bin/bash
# GPU box: N>1 bench rehearsal over gloo (2 ranks share the one GPU; W=4 on one GPU stalled in
# graph generation before any collective, so it is not run) + refreshed config timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS="${STEPS:-w2 configs}"
for s in $STEPS; do
  case $s in
    w2)
      MAXK_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29602 bench.py --gpus 2 --steps 5 --warmup 2 \
        --no-cpu-baseline --no-comparator --k-sweep "" > gpurun_out/rehearse_w2.json 2> gpurun_out/rehearse_w2.log || exit $?
      cat gpurun_out/rehearse_w2.json ;;
    configs)
      timeout -k 10 400 python -u tools/configs_time.py --out gpurun_out/configs.json 2>&1 | tee gpurun_out/configs.log || exit $? ;;
  esac
done
