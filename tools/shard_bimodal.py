"""Is the per-rank backward time of an 8-GPU shard bimodal per plan instance or per call?
(tooling, round 5). One rank's ShardedAggregation (as tools/shard_time.py builds it); its
backward timed R times on one plan, then P freshly built plans (new device allocations) timed
once each; also the same with the grad table and the gl copy re-allocated.

  python tools/shard_bimodal.py [--rank 3] [--plans 6] [--repeats 5]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-gnn_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import maxk_kernels as mk  # noqa: E402
from maxk_kernels import graphs  # noqa: E402
from maxk_kernels.dist import RowPartition, ShardedAggregation  # noqa: E402
from shard_time import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, default=3)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--plans", type=int, default=6)
    ap.add_argument("--repeats", type=int, default=5)
    ap.add_argument("--k", type=int, default=16)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n, e = graphs.DATASETS["reddit"]
    ptr = graphs.synthetic_ptr(n, e, seed=97, device=dev)
    d, k = 256, args.k
    h = graphs.features(n, d, seed=97, device=dev)
    g = graphs.features(n, d, seed=98, device=dev)
    sd, si = mk.maxk_forward(h, k, return_index=True)
    del h
    part = RowPartition(ptr, args.world)
    q = args.rank
    a, b = part.rows(q)
    idx_q = graphs.synthetic_rows(ptr, seed=97, rows=(a, b))
    val_q = graphs.sage_mean_values(ptr[a:b + 1], num_edges=idx_q.numel())
    shard = ShardedAggregation(part, q, ptr, idx_q, val_q, d, k, local_edges=True)
    for r in range(args.world):
        pos = part.table_positions(r, dev)
        ra, rb = part.rows(r)
        shard.table_data[pos] = sd[ra:rb]
        shard.table_index[pos] = si[ra:rb]
    ti = shard.table_index
    gl = g[a:b].contiguous()
    same = [timeit(lambda: shard.plan.backward(gl, ti, shard.grad_table)) for _ in range(args.repeats)]
    print(json.dumps({"rank": q, "same_plan_bwd_ms": same}), flush=True)
    fresh = []
    keep = []
    for _ in range(args.plans):
        plan = mk.GraphPlan(shard.plan._refs[0], shard.plan._refs[1], shard.plan._refs[2],
                            shard.plan.num_rows, shard.plan.num_edges, d, k,
                            num_cols=shard.plan.num_cols)
        out = torch.empty_like(shard.grad_table)
        fresh.append(timeit(lambda: plan.backward(gl, ti, out)))
        keep.append((plan, out))  # new addresses for every plan
    print(json.dumps({"rank": q, "fresh_plan_bwd_ms": fresh}), flush=True)
    again = [timeit(lambda: p.backward(gl, ti, o)) for p, o in keep]
    print(json.dumps({"rank": q, "fresh_plans_retimed_ms": again}), flush=True)
    # which allocation carries it: every plan with the first output, the first plan with
    # every output, and every plan with a fresh copy of the grad_out rows
    p0, o0 = keep[0]
    print(json.dumps({"rank": q, "plan_i_out_0": [timeit(lambda: p.backward(gl, ti, o0))
                                                   for p, _ in keep],
                      "plan_0_out_i": [timeit(lambda: p0.backward(gl, ti, o)) for _, o in keep],
                      "plan_0_fresh_gl": [timeit(lambda: p0.backward(gl.clone(), ti, o0))
                                          for _ in keep]}), flush=True)


if __name__ == "__main__":
    main()
