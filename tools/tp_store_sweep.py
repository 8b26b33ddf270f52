"""Two-pass backward workspace order (tooling): CSR-order stores + permuted column gathers
(bwd_tp_store=1) against column-order scattered stores + streamed columns (2).
  python tools/tp_store_sweep.py [--cases ogbn-products:32,ogbn-products:16,reddit:16]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-gnn_amd"))
import torch  # noqa: E402

import maxk_kernels as mk  # noqa: E402
from maxk_kernels import graphs  # noqa: E402


def timeit(fn, reps=10):
    for _ in range(2):
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
    ap.add_argument("--cases", default="ogbn-products:32,ogbn-products:16,reddit:16")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    for case in args.cases.split(","):
        ds, k = case.split(":")
        k = int(k)
        n, e = graphs.DATASETS[ds]
        ptr, idx = graphs.synthetic_csr(n, e, device=dev)
        val = graphs.sage_mean_values(ptr)
        e = idx.numel()
        h = graphs.features(n, 256, seed=97, device=dev)
        g = graphs.features(n, 256, seed=98, device=dev)
        sd, si = mk.maxk_forward(h, k, return_index=True)
        del h
        outs = {}
        for st in (1, 2):
            plan = mk.GraphPlan(ptr, idx, val, n, e, 256, k, options={"bwd_algo": 3, "bwd_tp_store": st})
            gr = torch.empty((n, k), device=dev)
            t = timeit(lambda: plan.backward(g, si, gr))
            outs[st] = gr.clone()
            print(json.dumps({"dataset": ds, "k": k, "bwd_tp_store": st, "bwd_ms": round(t, 4)}),
                  flush=True)
            del plan, gr
            torch.cuda.empty_cache()
        print(json.dumps({"dataset": ds, "k": k, "max_abs_diff": float((outs[1] - outs[2]).abs().max())}),
              flush=True)
        del ptr, idx, val, g, sd, si, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
