"""Per-rank device time of the row-partitioned path on ONE GPU (tooling): for W in 1,2,4,8
build each rank's rectangular plan exactly as maxk_kernels.dist does and time its SpGEMM
forward + SSpMM backward (no collectives), to see how the compute part strong-scales.

  python tools/shard_time.py [--k 16]
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
from maxk_kernels.dist import RowPartition  # noqa: E402


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
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--opts", default="[{}]", help="JSON list of plan option dicts to compare")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n, e = graphs.DATASETS[args.dataset]
    ptr, idx = graphs.synthetic_csr(n, e, device=dev)
    val = graphs.sage_mean_values(ptr)
    d, k = 256, args.k
    h = graphs.features(n, d, seed=97, device=dev)
    g = graphs.features(n, d, seed=98, device=dev)
    sd, si = mk.maxk_forward(h, k, return_index=True)
    for world, opts in [(int(w), o) for w in args.worlds.split(",") for o in json.loads(args.opts)]:
        part = RowPartition(ptr, world)
        m = part.max_rows
        td = torch.zeros((part.padded_rows, k), device=dev)
        tix = torch.zeros((part.padded_rows, k), dtype=torch.uint8, device=dev)
        for q in range(world):
            a, b = part.rows(q)
            td[q * m: q * m + b - a] = sd[a:b]
            tix[q * m: q * m + b - a] = si[a:b]
        worst = 0.0
        for q in (0, world - 1):
            a, b = part.rows(q)
            lp, li, lv = part.local_csr(ptr, idx, val, q)
            plan = mk.GraphPlan(lp, li, lv, b - a, li.numel(), d, k, num_cols=part.padded_rows,
                                options=opts)
            gl = g[a:b].contiguous()
            out = torch.empty((b - a, d), device=dev)
            gr = torch.empty((part.padded_rows, k), device=dev)
            tf = timeit(lambda: plan.forward(td, tix, out))
            tb = timeit(lambda: plan.backward(gl, tix, gr))
            worst = max(worst, tf + tb)
            print(json.dumps({"world": world, "opts": opts, "rank": q, "edges": li.numel(), "fwd_ms": tf,
                              "bwd_ms": tb, "info": plan.info()}), flush=True)
            del plan
        print(json.dumps({"world": world, "opts": opts, "compute_ms_max": worst,
                          "edges_per_s_compute_only": 2 * e / (worst * 1e-3)}), flush=True)


if __name__ == "__main__":
    main()
