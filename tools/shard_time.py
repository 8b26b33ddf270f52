"""Per-rank device time of the row-partitioned path on ONE GPU (tooling): for W in 1,2,4,8
build ranks' ShardedAggregation exactly as maxk_kernels.dist does, fill their gathered
tables (and statistics rows) as the all-gather would, and time the forward and backward
kernels alone (compute_forward / compute_backward: no collectives), to see how the compute
part strong-scales and what the variants cost:

  stats   : the forward reads the W gathered statistics pairs (default) / scans the table
  split   : the local-columns-first split (two plans per rank) / one plan

  python tools/shard_time.py [--k 16] [--worlds 1,2,4,8] [--variants '[...]']
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
    ap.add_argument("--variants", default='[{"split": false, "stats": true}, '
                                          '{"split": false, "stats": false}, '
                                          '{"split": true, "stats": true}]')
    ap.add_argument("--opts", default="{}", help="plan options (JSON dict)")
    ap.add_argument("--phases", default="1", help="column phases to try (comma list; > 1 "
                    "drops the statistics row)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n, e = graphs.DATASETS[args.dataset]
    ptr, idx = graphs.synthetic_csr(n, e, device=dev)
    val = graphs.sage_mean_values(ptr)
    d, k = 256, args.k
    h = graphs.features(n, d, seed=97, device=dev)
    g = graphs.features(n, d, seed=98, device=dev)
    sd, si = mk.maxk_forward(h, k, return_index=True)
    del h
    opts = json.loads(args.opts)
    for world, phases in [(int(w), int(p)) for w in args.worlds.split(",")
                          for p in args.phases.split(",")]:
        part = RowPartition(ptr, world, phases=phases)
        for var in json.loads(args.variants):
            worst = 0.0
            for q in sorted({0, world - 1}):
                shard = ShardedAggregation(part, q, ptr, idx, val, d, k, plan_options=opts,
                                           split=var["split"])
                a, b = part.rows(q)
                shard._stage(sd[a:b], si[a:b])          # send buffers + this rank's stats row
                shard.table_data.zero_()                # spare rows: zeros, as gathered
                shard.table_index.zero_()
                for r in range(world):                  # the all-gather, emulated
                    ra, rb = part.rows(r)
                    pos = part.table_positions(r, dev)
                    shard.table_data[pos] = sd[ra:rb]
                    shard.table_index[pos] = si[ra:rb]
                    if shard.stats:
                        mk.cbsr_stats(sd[ra:rb], si[ra:rb],
                                      out=shard.stats_words(shard.table_index,
                                                            part.stats_position(r)))
                shard.stats = shard.stats and var["stats"]
                gl = g[a:b].contiguous()
                tf = timeit(shard.compute_forward)
                tb = timeit(lambda: shard.compute_backward(gl))
                worst = max(worst, tf + tb)
                print(json.dumps({"world": world, "phases": phases, **var, "opts": opts, "rank": q,
                                  "edges": int(shard.ptr[-1]), "fwd_ms": tf, "bwd_ms": tb,
                                  "plans": [p.info() for p in shard.plans]}), flush=True)
                del shard
            print(json.dumps({"world": world, "phases": phases, **var, "opts": opts,
                              "compute_ms_max": worst,
                              "edges_per_s_compute_only": 2 * e / (worst * 1e-3)}), flush=True)


if __name__ == "__main__":
    main()
