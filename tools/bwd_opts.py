"""Backward plan-option A/B on a dataset-shaped synthetic graph (tooling): HIP-event ms of the
SSpMM backward call per option set, interleaved over several rounds (so box drift hits every
variant alike), with the plan's task count and the largest deviation from the first set.
  python tools/bwd_opts.py --k 16 --opts '[{}, {"bwd_order": 2}]' [--dataset reddit] [--rounds 3]"""
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
    ap.add_argument("--dataset", default="reddit")
    ap.add_argument("--opts", default="[{}]")
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n, e = graphs.DATASETS[args.dataset]
    ptr = graphs.synthetic_ptr(n, e, seed=97, device=dev)
    idx = graphs.synthetic_rows(ptr, seed=97)
    e = idx.numel()
    val = graphs.sage_mean_values(ptr, num_edges=e)
    h = graphs.features(n, 256, seed=97, device=dev)
    _, si = mk.maxk_forward(h, args.k, return_index=True)
    del h
    g = graphs.features(n, 256, seed=98, device=dev)
    sets = json.loads(args.opts)
    plans = [mk.GraphPlan(ptr, idx, val, n, e, 256, args.k, options=o) for o in sets]
    outs = [torch.empty((n, args.k), device=dev) for _ in sets]
    times = [[] for _ in sets]
    for _ in range(args.rounds):
        for i, p in enumerate(plans):
            times[i].append(timeit(lambda: p.backward(g, si, outs[i])))
    for i, o in enumerate(sets):
        dev_max = float(((outs[i] - outs[0]).abs() / (outs[0].abs() + 1e-3)).max())
        t = sorted(times[i])
        print(json.dumps({"dataset": args.dataset, "k": args.k, "opts": o,
                          "bwd_ms": round(t[len(t) // 2], 4), "bwd_ms_all": [round(x, 4) for x in times[i]],
                          "tasks": plans[i].info()["bwd_tasks"], "max_rel_dev": dev_max,
                          "dense_edges": plans[i].info().get("bwd_dense_edges"),
                          "dense_runs": plans[i].info().get("bwd_dense_runs")}), flush=True)


if __name__ == "__main__":
    main()
