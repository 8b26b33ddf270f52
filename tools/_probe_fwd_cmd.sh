# GPU box: forward LDS-update probes (tools/probe_fwd_build.py) at k = 16/32/64, full table and an
# L2-resident 4096-node window (tools/fwd_locality.py).
for lib in product tools/libmaxk_probe_nolds.so tools/libmaxk_probe_u64.so tools/libmaxk_probe_rmw.so; do
  for k in 16 32 64; do
    if [ "$lib" = product ]; then unset MAXK_HIP_LIB; else export MAXK_HIP_LIB=$PWD/$lib; fi
    timeout -k 10 150 python -u tools/fwd_locality.py --k $k --windows 0,4096 --fwd-only >> gpurun_out/probe_fwd.jsonl 2>>gpurun_out/probe_fwd.err || exit $?
  done
done
cat gpurun_out/probe_fwd.jsonl
