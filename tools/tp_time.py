"""Two-pass backward timing on the ogbn-products-shaped graph (tooling): the SSpMM backward
call at k (default 32) with the default plan, HIP events, one JSON line. Run under
rocprofv3 --kernel-trace --stats for the row / column pass split.
  python tools/tp_time.py [--k 32] [--opts '{}']"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-gnn_amd"))
import torch  # noqa: E402

import maxk_kernels as mk  # noqa: E402
from maxk_kernels import graphs  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=32)
    ap.add_argument("--dataset", default="ogbn-products")
    ap.add_argument("--opts", default="{}")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n, e = graphs.DATASETS[args.dataset]
    ptr, idx = graphs.bench_csr(args.dataset, device=dev)
    val = graphs.sage_mean_values(ptr)
    h = graphs.features(n, 256, seed=97, device=dev)
    g = graphs.features(n, 256, seed=98, device=dev)
    sd, si = mk.maxk_forward(h, args.k, return_index=True)
    del h
    plan = mk.GraphPlan(ptr, idx, val, n, idx.numel(), 256, args.k, options=json.loads(args.opts))
    gs = plan.backward(g, si)
    ref = gs.clone()
    for _ in range(2):
        plan.backward(g, si, gs)
    s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        plan.backward(g, si, gs)
    t.record()
    t.synchronize()
    dev_ = float(((gs - ref).abs() / (ref.abs() + 1e-3)).max())
    print(json.dumps({"dataset": args.dataset, "k": args.k, "opts": args.opts,
                      "bwd_ms": s.elapsed_time(t) / 10, "tp_rows": plan.info().get("bwd_algo"),
                      "rerun_max_rel_dev": dev_}), flush=True)


if __name__ == "__main__":
    main()
