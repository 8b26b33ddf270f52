"""Supplementary measurement (tooling): the SpGEMM forward and SSpMM backward on
Reddit-sized graphs with and without column locality, for a list of plan option sets.

  uniform    : graphs.synthetic_csr, the BASELINE workload (uniform random columns)
  community  : graphs.community_csr, 41 communities, p_in 0.76, in ID order (locality visible)
  shuffled   : the same community graph under a random relabelling (locality hidden)

Prints one JSON line per (graph, k, option set): E, plan build s, fwd/bwd ms (HIP events,
median of 5 x 10), the algorithmic-byte roofline fraction of each kernel, and the plan info.
  python tools/locality_graphs.py [--k 16,32] [--opts '[{}, {"col_order": 2}]']"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-gnn_amd"))
import torch  # noqa: E402

import maxk_kernels as mk  # noqa: E402
from maxk_kernels import graphs  # noqa: E402


def timeit(fn, reps=10, rounds=5):
    fn()
    ts = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) / reps)
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", default="16")
    ap.add_argument("--graphs", default="uniform,community,shuffled")
    ap.add_argument("--opts", default="[{}]", help="JSON option dict or list of dicts")
    ap.add_argument("--which", default="both", choices=["fwd", "bwd", "both"])
    ap.add_argument("--dataset", default="reddit")
    args = ap.parse_args()
    opt_sets = json.loads(args.opts)
    if isinstance(opt_sets, dict):
        opt_sets = [opt_sets]
    dev = torch.device("cuda:0")
    n, e0 = graphs.DATASETS[args.dataset]
    d = 256
    h = graphs.features(n, d, seed=97, device=dev)
    g = graphs.features(n, d, seed=98, device=dev)
    for name in args.graphs.split(","):
        if name == "uniform":
            ptr, idx = graphs.synthetic_csr(n, e0, device=dev)
        else:
            ptr, idx = graphs.community_csr(n, e0, shuffle=name == "shuffled", device=dev)
        val = graphs.sage_mean_values(ptr)
        e = idx.numel()
        for k in [int(x) for x in args.k.split(",")]:
            sd, si = mk.maxk_forward(h, k, return_index=True)
            for opts in opt_sets:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                plan = mk.GraphPlan(ptr, idx, val, n, e, d, k, options=opts)
                torch.cuda.synchronize()
                build_s = time.perf_counter() - t0
                tf = tb = None
                if args.which in ("fwd", "both"):
                    out = plan.forward(sd, si)
                    tf = timeit(lambda: plan.forward(sd, si, out))
                if args.which in ("bwd", "both"):
                    gr = plan.backward(g, si)
                    tb = timeit(lambda: plan.backward(g, si, gr))
                fb = 4 * (n + 1) + 8 * e + 5 * k * n + 4 * d * n
                bb = 4 * (n + 1) + 8 * e + 4 * d * n + k * n + 4 * k * n
                print(json.dumps({
                    "graph": name, "k": k, "opts": opts, "num_edges": e,
                    "build_s": round(build_s, 3),
                    "fwd_ms": None if tf is None else round(tf, 4),
                    "bwd_ms": None if tb is None else round(tb, 4),
                    "fwd_roofline_frac": None if tf is None else fb / (tf * 1e-3) / 8e12,
                    "bwd_roofline_frac": None if tb is None else bb / (tb * 1e-3) / 8e12,
                    "info": plan.info()}), flush=True)
                del plan
            del sd, si
        del ptr, idx, val


if __name__ == "__main__":
    main()
