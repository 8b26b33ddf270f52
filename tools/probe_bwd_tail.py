"""Per-work-group durations of one column-block backward launch (tooling, round 5; build
tools/libprobe_bwd_tail.so as tools/probe_bwd_tail.hip says and run with
MAXK_HIP_LIB=tools/libprobe_bwd_tail.so). For the Reddit bench graph at k (and an 8-GPU row
shard), one JSON line per case: the launch's span (first start to last end), the mean / p50 /
p90 / max work-group duration, and the idle share of the span, 1 - sum(durations) / (span x
work-groups running at once).

  MAXK_HIP_LIB=tools/libprobe_bwd_tail.so python tools/probe_bwd_tail.py [--k 16]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-gnn_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import maxk_kernels as mk  # noqa: E402
from maxk_kernels import graphs  # noqa: E402
from maxk_kernels._lib import lib  # noqa: E402
from maxk_kernels.dist import RowPartition, ShardedAggregation  # noqa: E402

lib.probe_bwd_clocks.restype = ctypes.c_int
lib.probe_bwd_clocks.argtypes = [ctypes.c_void_p, ctypes.c_int]


def clocks(n):
    buf = np.zeros(2 * n, dtype=np.uint64)
    rc = lib.probe_bwd_clocks(buf.ctypes.data, n)
    assert rc == n, rc
    return buf[:n].astype(np.int64), buf[n:].astype(np.int64)


def report(name, plan, fn, reps=5):
    n = plan.info()["bwd_tasks"]
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    rows = []
    for _ in range(reps):
        fn()
        s, e = clocks(n)
        d = (e - s) * 10.0 / 1e3             # us (100 MHz)
        span = (e.max() - s.min()) * 10.0 / 1e3
        conc = min(n, cus)
        rows.append({"span_us": span, "mean_us": float(d.mean()), "p50_us": float(np.median(d)),
                     "p90_us": float(np.percentile(d, 90)), "max_us": float(d.max()),
                     "min_us": float(d.min()),
                     "idle_share": float(1 - d.sum() / (span * conc))})
    if os.environ.get("PROBE_DUMP"):   # raw clocks of the last launch, with the plan's tasks
        np.savez(os.path.join(os.environ["PROBE_DUMP"], name.replace(" ", "_").replace("=", "") + ".npz"),
                 start=s, end=e)
    best = min(rows, key=lambda r: r["span_us"])
    worst = max(rows, key=lambda r: r["span_us"])
    print(json.dumps({"case": name, "tasks": n, "best": best, "worst": worst}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=16)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n, _ = graphs.DATASETS["reddit"]
    ptr, idx = graphs.bench_csr("reddit", device=dev)
    e = idx.numel()
    val = graphs.sage_mean_values(ptr, num_edges=e)
    d, k = 256, args.k
    h = graphs.features(n, d, seed=97, device=dev)
    g = graphs.features(n, d, seed=98, device=dev)
    sd, si = mk.maxk_forward(h, k, return_index=True)
    plan = mk.GraphPlan(ptr, idx, val, n, e, d, k)
    out = torch.empty(n, k, device=dev)
    report(f"reddit k={k}", plan, lambda: plan.backward(g, si, out))
    del plan, out
    # an 8-GPU row shard (rank 3), as tools/shard_time.py builds it
    ptr8 = graphs.synthetic_ptr(n, e, seed=97, device=dev)
    part = RowPartition(ptr8, 8)
    a, b = part.rows(3)
    idx_q = graphs.synthetic_rows(ptr8, seed=97, rows=(a, b))
    val_q = graphs.sage_mean_values(ptr8[a:b + 1], num_edges=idx_q.numel())
    shard = ShardedAggregation(part, 3, ptr8, idx_q, val_q, d, k, local_edges=True)
    for r in range(8):
        pos = part.table_positions(r, dev)
        ra, rb = part.rows(r)
        shard.table_data[pos] = sd[ra:rb]
        shard.table_index[pos] = si[ra:rb]
    gl = g[a:b].contiguous()
    report(f"8-GPU shard rank 3 k={k}", shard.plan,
           lambda: shard.plan.backward(gl, shard.table_index, shard.grad_table))


if __name__ == "__main__":
    main()
