"""Forward accumulation sweep (tooling): fixed point (fwd_fixed=1) against f64 atomics
(fwd_fixed=2) on the Reddit-shaped graph, per k and per forward layout; HIP-event time of
plan.forward (the stats pass included) and the max deviation between the two paths.
  python tools/fwd_fixed_sweep.py [--k 8,16,24,32,64] [--opts '{}']"""
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
    ap.add_argument("--k", default="8,16,24,32,64")
    ap.add_argument("--opts", default="{}")
    ap.add_argument("--dataset", default="reddit")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n, e = graphs.DATASETS[args.dataset]
    ptr, idx = graphs.synthetic_csr(n, e, device=dev)
    val = graphs.sage_mean_values(ptr)
    e = idx.numel()
    h = graphs.features(n, 256, seed=97, device=dev)
    for k in [int(x) for x in args.k.split(",")]:
        sd, si = mk.maxk_forward(h, k, return_index=True)
        res = {}
        outs = {}
        for fixed in (1, 2):
            opts = dict(json.loads(args.opts), fwd_fixed=fixed)
            plan = mk.GraphPlan(ptr, idx, val, n, e, 256, k, options=opts)
            out = torch.empty((n, 256), device=dev)
            res[fixed] = timeit(lambda: plan.forward(sd, si, out))
            outs[fixed] = out.clone()
            del plan
        dev_max = float(((outs[1] - outs[2]).abs() / (outs[2].abs() + 1e-6)).max())
        print(json.dumps({"dataset": args.dataset, "k": k, "opts": args.opts,
                          "fixed_ms": round(res[1], 4), "f64_ms": round(res[2], 4),
                          "max_rel_dev": dev_max}), flush=True)


if __name__ == "__main__":
    main()
