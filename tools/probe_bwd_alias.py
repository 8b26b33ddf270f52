"""Drives tools/probe_bwd_alias.hip (tooling): packed-backward time on the Reddit-shaped graph
when grad_out row r is read as row r % mod (working sets from the whole grad_out down to a
few MB), to see whether L2 residency of the gathered rows moves the backward.
  python tools/probe_bwd_alias.py [--k 16] [--mods 0,65536,8192,2048]"""
import argparse
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "spgemm-gnn_amd"))
import torch  # noqa: E402

import maxk_kernels as mk  # noqa: E402
from maxk_kernels import graphs  # noqa: E402

SO = os.path.join(HERE, "libprobe_bwd_alias.so")


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--mods", default="0,65536,16384,4096,2048")
    args = ap.parse_args()
    lib = ctypes.CDLL(SO)
    lib.probe_alias_rows.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    n, e = graphs.DATASETS["reddit"]
    ptr, idx = graphs.synthetic_csr(n, e, device=dev)
    val = graphs.sage_mean_values(ptr)
    h = graphs.features(n, 256, seed=97, device=dev)
    g = graphs.features(n, 256, seed=98, device=dev)
    sd, si = mk.maxk_forward(h, args.k, return_index=True)
    gs = torch.empty_like(sd)
    for mod in [int(m) for m in args.mods.split(",")]:
        plan = mk.GraphPlan(ptr, idx, val, n, e, 256, args.k)
        if mod:
            rc = lib.probe_alias_rows(plan.handle, mod,
                                      ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
            assert rc == 0, rc
        t = timeit(lambda: plan.backward(g, si, gs))
        print(json.dumps({"k": args.k, "mod_rows": mod, "working_set_MB": (mod or n) * 1024 / 1e6,
                          "bwd_ms": round(t, 4)}), flush=True)
        del plan


if __name__ == "__main__":
    main()
