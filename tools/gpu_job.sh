#!/bin/bash
# One GPU job (tooling): run named steps in order, each under its own time limit, with its
# output in gpurun_out/<name>.log. A fault, abort, segfault or time limit ends the job, so
# nothing else touches the GPU after it; test failures (pytest exit 1) do not.
#
#   bash tools/gpu_job.sh 'name|seconds|command' ['name|seconds|command' ...]
#
# e.g. gpurun -- bash tools/gpu_job.sh \
#        'tests|600|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread' \
#        'bench|300|python -u bench.py --steps 20'
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%|*}
  rest=${spec#*|}
  secs=${rest%%|*}
  cmd=${rest#*|}
  echo "== $name (${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 4 "gpurun_out/$name.log"
  case $rc in
    0|1|5) ;;
    *) echo "== stopping after $name (rc=$rc)"; exit "$rc" ;;
  esac
done
