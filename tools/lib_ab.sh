#!/bin/bash
# A/B of two builds of libmaxk_hip.so on the default plans (tooling): the candidate in-tree
# library vs tools/ab/libmaxk_hip_base.so (MAXK_HIP_LIB), alternating processes, Reddit
# forward and backward at each k; one JSON line per run with "lib".
#   bash tools/lib_ab.sh [ks] [rounds]
KS=${1:-"8 16 32 64"}
R=${2:-3}
for r in $(seq 1 $R); do
  for lib in base cand; do
    for k in $KS; do
      if [ $lib = base ]; then export MAXK_HIP_LIB="$PWD/tools/ab/libmaxk_hip_base.so"; else unset MAXK_HIP_LIB; fi
      timeout -k 10 120 python -u tools/bwd_opts.py --k $k --rounds 1 --opts '[{}]' | sed "s/^{/{\"lib\": \"$lib\", /" || exit 1
      timeout -k 10 120 python -u tools/fwd_opts_sweep.py --k $k --rounds 1 --opts '[{}]' | sed "s/^{/{\"lib\": \"$lib\", /" || exit 1
    done
  done
done
