"""BASELINE.json config 1 (CPU plumbing, no GPU): the DGL-semantics aggregation of a GraphSAGE
layer on a Flickr-shaped graph, hidden 64, ReLU input, timed with the oracle's C/OpenMP
dense CSR SpMM (update_all(copy_u, mean): forward A_mean @ X and its backward A_mean^T @ G)
on this machine's cores. Prints one JSON line.

  python tools/cpu_config1.py [--reps 10] [--threads N]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-gnn_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from maxk_kernels import graphs  # noqa: E402
from oracle import oracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--dataset", default="flickr")
    ap.add_argument("--hidden", type=int, default=64)
    args = ap.parse_args()
    n, e = graphs.DATASETS[args.dataset]
    ptr, idx = graphs.synthetic_csr(n, e, seed=97)
    val = graphs.sage_mean_values(ptr).numpy()
    p, ix = ptr.numpy(), idx.numpy()
    x = np.maximum(graphs.features(n, args.hidden, seed=97).numpy(), 0.0)   # ReLU input
    g = graphs.features(n, args.hidden, seed=98).numpy()
    # transposed graph for the backward A^T G
    rows = np.repeat(np.arange(n, dtype=np.int32), np.diff(p))
    order = np.argsort(ix, kind="stable")
    pt = np.zeros(n + 1, np.int32)
    pt[1:] = np.cumsum(np.bincount(ix, minlength=n))
    it, vt = rows[order], val[order]
    y = np.zeros((n, args.hidden), np.float32)
    for _ in range(2):   # warm-up
        oracle.dense_spmm(p, ix, val, x, out=y)
        oracle.dense_spmm(pt, it, vt, g, out=y)
    tf, tb = [], []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        oracle.dense_spmm(p, ix, val, x, out=y)
        t1 = time.perf_counter()
        oracle.dense_spmm(pt, it, vt, g, out=y)
        t2 = time.perf_counter()
        tf.append(t1 - t0)
        tb.append(t2 - t1)
    tf, tb = float(np.median(tf)), float(np.median(tb))
    cpu = "unknown"
    for line in open("/proc/cpuinfo"):
        if line.startswith("model name"):
            cpu = line.split(":", 1)[1].strip()
            break
    print(json.dumps({
        "config": f"{args.dataset} GraphSAGE hidden={args.hidden} ReLU, DGL-semantics CPU SpMM "
                  "(oracle C/OpenMP; synthetic graph, seed 97)",
        "num_nodes": n, "num_edges": int(p[-1]), "fwd_ms_median": tf * 1e3,
        "bwd_ms_median": tb * 1e3, "edges_per_s": 2 * int(p[-1]) / (tf + tb),
        "threads": oracle.num_threads(), "cpu_model": cpu, "host_cpus": os.cpu_count(),
        "reps": args.reps}))


if __name__ == "__main__":
    main()
