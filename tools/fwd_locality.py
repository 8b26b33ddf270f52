"""Upper bound of what column locality buys the SpGEMM forward (tooling): Reddit's N, E and
degree sequence with the columns of every edge folded into a window of W nodes
(col % W), so the gathered CBSR table is W x 128 B instead of N x 128 B. Prints one JSON
line per window: forward ms (HIP events) and the L2-resident fraction of the table.

  python tools/fwd_locality.py [--windows 0,131072,32768,8192]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-gnn_amd"))
import torch  # noqa: E402

import maxk_kernels as mk  # noqa: E402
from maxk_kernels import graphs  # noqa: E402


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
    ap.add_argument("--windows", default="0,131072,32768,8192")
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--opts", default="{}")
    ap.add_argument("--fwd-only", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n, e = graphs.DATASETS["reddit"]
    ptr, idx = graphs.synthetic_csr(n, e, device=dev)
    val = graphs.sage_mean_values(ptr)
    h = graphs.features(n, 256, seed=97, device=dev)
    g = graphs.features(n, 256, seed=98, device=dev)
    sd, si = mk.maxk_forward(h, args.k, return_index=True)
    for w in [int(x) for x in args.windows.split(",")]:
        ix = idx if w == 0 else (idx % w)
        if w:
            # keep each row's columns sorted (the plan expects CSR order; duplicates are fine)
            rows = torch.repeat_interleave(torch.arange(n, device=dev), (ptr[1:] - ptr[:-1]).long())
            key = rows * n + ix.long()
            ix = (torch.sort(key).values - rows * n).to(torch.int32)
        plan = mk.GraphPlan(ptr, ix, val, n, e, 256, args.k, options=json.loads(args.opts))
        out = torch.empty((n, 256), device=dev)
        gr = torch.empty((n, args.k), device=dev)
        tf = timeit(lambda: plan.forward(sd, si, out))
        tb = None if args.fwd_only else timeit(lambda: plan.backward(g, si, gr))
        print(json.dumps({"window": w, "table_MB": (w or n) * 128 / 1e6, "fwd_ms": tf,
                          "bwd_ms": tb, "opts": args.opts,
                          "lib": os.path.basename(os.environ.get("MAXK_HIP_LIB", "libmaxk_hip.so"))}), flush=True)
        del plan


if __name__ == "__main__":
    main()
