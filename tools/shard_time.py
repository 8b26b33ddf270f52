"""Per-rank device time of the row-partitioned path on ONE GPU (tooling): for W in 1,2,4,8
build ranks' ShardedAggregation exactly as bench.py does (each rank generates its rows of the
bench graph), fill their gathered record tables (and statistics pairs) as the one all-gather
would, and time the forward and backward kernels alone (compute_forward / compute_backward: no
collectives), to see how the compute part strong-scales:

  records : the forward gathers the all-gathered interleaved records in place (default);
            "tables": the same plan over two contiguous tables (round 3's exchange layout,
            packed per call or gathered as two tables)

  python tools/shard_time.py [--k 16] [--worlds 1,2,4,8] [--opts '{}'] [--layouts records,tables]
                            [--all-ranks]
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
from maxk_kernels.dist import RowPartition, ShardedAggregation  # noqa: E402


def timeit(fn, reps=20, rounds=3):
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
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--dataset", default="reddit")
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--opts", default="{}", help="plan options (JSON dict)")
    ap.add_argument("--layouts", default="records,tables")
    ap.add_argument("--all-ranks", action="store_true", help="time every rank, not 0 and W-1")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n, e = graphs.DATASETS[args.dataset]
    ptr = graphs.synthetic_ptr(n, e, seed=97, device=dev)
    d, k = 256, args.k
    h = graphs.features(n, d, seed=97, device=dev)
    g = graphs.features(n, d, seed=98, device=dev)
    sd, si = mk.maxk_forward(h, k, return_index=True)
    del h
    opts = json.loads(args.opts)
    for world in [int(w) for w in args.worlds.split(",")]:
        part = RowPartition(ptr, world)
        for layout in args.layouts.split(","):
            worst = 0.0
            for q in (range(world) if args.all_ranks else sorted({0, world - 1})):
                a, b = part.rows(q)
                idx_q = graphs.synthetic_rows(ptr, seed=97, rows=(a, b))
                val_q = graphs.sage_mean_values(ptr[a:b + 1], num_edges=idx_q.numel())
                shard = ShardedAggregation(part, q, ptr, idx_q, val_q, d, k, plan_options=opts,
                                           local_edges=True)
                shard._stage(sd[a:b], si[a:b])          # send records + this rank's stats pair
                for r in range(world):                  # the all-gather, emulated
                    ra, rb = part.rows(r)
                    pos = part.table_positions(r, dev)
                    shard.table_data[pos] = sd[ra:rb]
                    shard.table_index[pos] = si[ra:rb]
                    mk.cbsr_stats(sd[ra:rb], si[ra:rb], out=shard.table_rec.view(
                        torch.int32)[part.stats_position(r), :2])
                td, ti = shard.table_data, shard.table_index
                if layout == "tables":                  # two contiguous tables instead
                    td, ti = td.contiguous(), ti.contiguous()
                gl = g[a:b].contiguous()
                tf = timeit(lambda: shard.plan.forward(td, ti, stats=shard._stats_all))
                tb = timeit(lambda: shard.plan.backward(gl, ti, shard.grad_table))
                worst = max(worst, tf + tb)
                print(json.dumps({"world": world, "layout": layout, "opts": opts, "rank": q,
                                  "edges": int(shard.ptr[-1]), "fwd_ms": tf, "bwd_ms": tb,
                                  "plan": shard.plan.info()}), flush=True)
                del shard
            print(json.dumps({"world": world, "layout": layout, "opts": opts,
                              "compute_ms_max": worst,
                              "edges_per_s_compute_only": 2 * e / (worst * 1e-3)}), flush=True)


if __name__ == "__main__":
    main()
