"""Launch-overhead check (tooling): the SpGEMM forward + SSpMM backward step timed as eager
launches and replayed from a captured HIP graph (torch.cuda.CUDAGraph over the ctypes
launches, which all go to the capture stream), on the Reddit-shaped graph at W = 1 and on one
rank's shard at W = 8 (tools/shard_time.py's emulated gather).
  python tools/graph_time.py [--k 16] [--worlds 1,8]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-gnn_amd"))
import torch  # noqa: E402

import maxk_kernels as mk  # noqa: E402
from maxk_kernels import graphs  # noqa: E402
from maxk_kernels.dist import RowPartition, ShardedAggregation  # noqa: E402


def timeit(fn, reps=50, rounds=5):
    fn()
    torch.cuda.synchronize()
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


def captured(fn):
    fn()  # warm: plans, workspaces, LDS attributes
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g.replay


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--worlds", default="1,8")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n, e = graphs.DATASETS["reddit"]
    ptr, idx = graphs.bench_csr("reddit", device=dev)
    val = graphs.sage_mean_values(ptr)
    d, k = 256, args.k
    h = graphs.features(n, d, seed=97, device=dev)
    g = graphs.features(n, d, seed=98, device=dev)
    sd, si = mk.maxk_forward(h, k, return_index=True)
    for world in [int(w) for w in args.worlds.split(",")]:
        if world == 1:
            plan = mk.GraphPlan(ptr, idx, val, n, e, d, k)
            out = torch.empty((n, d), device=dev)
            gs = torch.empty((n, k), device=dev)

            def step():
                plan.forward(sd, si, out)
                plan.backward(g, si, gs)
        else:
            part = RowPartition(ptr, world)
            q = world - 1
            shard = ShardedAggregation(part, q, ptr, idx, val, d, k)
            a, b = part.rows(q)
            shard._stage(sd[a:b], si[a:b])
            shard.table_data.zero_()
            shard.table_index.zero_()
            for r in range(world):
                ra, rb = part.rows(r)
                pos = part.table_positions(r, dev)
                shard.table_data[pos] = sd[ra:rb]
                shard.table_index[pos] = si[ra:rb]
                mk.cbsr_stats(sd[ra:rb], si[ra:rb],
                              out=shard.stats_words(shard.table_index, part.stats_position(r)))
            gl = g[a:b].contiguous()

            def step():
                shard.compute_forward()
                shard.compute_backward(gl)
        t_eager = timeit(step)
        t_graph = timeit(captured(step))
        print(json.dumps({"world": world, "k": k, "eager_ms": round(t_eager, 4),
                          "graph_ms": round(t_graph, 4),
                          "saved_pct": round(100 * (1 - t_graph / t_eager), 2)}), flush=True)


if __name__ == "__main__":
    main()
