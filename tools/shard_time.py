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
    ap.add_argument("--phases", default="1", help="column phases to compare, e.g. 1,2")
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
    for world, phases, opts in [(int(w), int(ph), o) for w in args.worlds.split(",")
                                for ph in args.phases.split(",") for o in json.loads(args.opts)]:
        part = RowPartition(ptr, world, phases=phases)
        td = torch.zeros((part.padded_rows, k), device=dev)
        tix = torch.zeros((part.padded_rows, k), dtype=torch.uint8, device=dev)
        for q in range(world):
            a, b = part.rows(q)
            pos = part.table_positions(q, dev)
            td[pos] = sd[a:b]
            tix[pos] = si[a:b]
        nc = part.phase_cols
        worst = 0.0
        for q in (0, world - 1):
            a, b = part.rows(q)
            lp, li, lv = part.local_csr(ptr, idx, val, q)
            plans = []
            for ph in range(phases):
                pp, pi, pv = part.phase_csr(lp, li, lv, ph)
                plans.append(mk.GraphPlan(pp, pi, pv, b - a, pi.numel(), d, k, num_cols=nc,
                                          options=opts))
            gl = g[a:b].contiguous()
            out = torch.empty((b - a, d), device=dev)
            gr = torch.empty((part.padded_rows, k), device=dev)

            def fwd():
                for ph, pl in enumerate(plans):
                    pl.forward(td[ph * nc:(ph + 1) * nc], tix[ph * nc:(ph + 1) * nc], out,
                               accumulate=ph > 0)

            def bwd():
                for ph, pl in enumerate(plans):
                    pl.backward(gl, tix[ph * nc:(ph + 1) * nc], gr[ph * nc:(ph + 1) * nc])

            tf = timeit(fwd)
            tb = timeit(bwd)
            worst = max(worst, tf + tb)
            print(json.dumps({"world": world, "phases": phases, "opts": opts, "rank": q,
                              "edges": li.numel(), "fwd_ms": tf, "bwd_ms": tb,
                              "info": plans[0].info()}), flush=True)
            del plans
        print(json.dumps({"world": world, "phases": phases, "opts": opts,
                          "compute_ms_max": worst,
                          "edges_per_s_compute_only": 2 * e / (worst * 1e-3)}), flush=True)


if __name__ == "__main__":
    main()
