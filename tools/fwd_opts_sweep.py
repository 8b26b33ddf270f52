"""Forward plan-option sweep on the Reddit-shaped graph (tooling): HIP-event ms per
option set (interleaved rounds, median), with the plan's task count.
  python tools/fwd_opts_sweep.py --k 16 --opts '[{}, {"fwd_rot_rate": 200}]'"""
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
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--dataset", default="reddit")
    ap.add_argument("--opts", default='[{}]')
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n, e = graphs.DATASETS[args.dataset]
    ptr, idx = graphs.bench_csr(args.dataset, device=dev)
    val = graphs.sage_mean_values(ptr)
    e = idx.numel()
    h = graphs.features(n, 256, seed=97, device=dev)
    sd, si = mk.maxk_forward(h, args.k, return_index=True)
    sets = json.loads(args.opts)
    plans = [mk.GraphPlan(ptr, idx, val, n, e, 256, args.k, options=o) for o in sets]
    outs = [torch.empty((n, 256), device=dev) for _ in sets]
    times = [[] for _ in sets]
    for _ in range(args.rounds):  # interleaved, so box drift hits every set alike
        for i, plan in enumerate(plans):
            times[i].append(timeit(lambda: plan.forward(sd, si, outs[i])))
    for i, opts in enumerate(sets):
        t = sorted(times[i])
        dev_max = float(((outs[i] - outs[0]).abs() / (outs[0].abs() + 1e-3)).max())
        print(json.dumps({"k": args.k, "opts": opts, "fwd_ms": round(t[len(t) // 2], 4),
                          "fwd_ms_all": [round(x, 4) for x in times[i]],
                          "tasks": plans[i].info()["fwd_tasks"], "max_rel_dev": dev_max}),
              flush=True)

if __name__ == "__main__":
    main()
