# GPU box: backward LDS-update probes (tools/probe_fwd_build.py bnolds bu32) at k = 8..64
for lib in product tools/libmaxk_probe_bnolds.so tools/libmaxk_probe_bu32.so; do
  for k in 8 16 32 64; do
    if [ "$lib" = product ]; then unset MAXK_HIP_LIB; else export MAXK_HIP_LIB=$PWD/$lib; fi
    timeout -k 10 150 python -u tools/fwd_locality.py --k $k --windows 0 >> gpurun_out/probe_bwd.jsonl 2>>gpurun_out/probe_bwd.err || exit $?
  done
done
cat gpurun_out/probe_bwd.jsonl
