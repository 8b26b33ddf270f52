#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Stops at the first step that crashes, times out or faults (exit codes other than 0/1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
STEPS="${STEPS:-tests smoke bench prof}"
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/gpu_tests.log" 2>&1; rc=$?
      tail -3 "$OUT/gpu_tests.log"; ok $rc || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
      tail -1 "$OUT/smoke.log"; ok $rc || exit $rc ;;
    bench)
      timeout -k 10 900 python bench.py ${BENCH_ARGS} > "$OUT/bench.json" 2> "$OUT/bench.log"; rc=$?
      cat "$OUT/bench.json"; tail -5 "$OUT/bench.log"; [ $rc -eq 0 ] || exit $rc ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats \
        -d "$OUT/prof" -o bench --output-format csv -- \
        python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-comparator --k-sweep "" ${BENCH_ARGS} \
        > "$OUT/prof_bench.json" 2> "$OUT/prof.log"); rc=$?
      tail -3 "$OUT/prof.log"; [ $rc -eq 0 ] || exit $rc
      find "$OUT/prof" -name "*kernel_stats.csv" | head -3 ;;
  esac
done
