"""Device time of the BASELINE.json configs besides the headline (tooling; one MI355X).

  python tools/configs_time.py [--out gpurun_out/configs.json]

* config 2: Reddit SpGEMM forward only, k=16, against rocSPARSE CSR SpMM on the dense MaxK
  output (the same numbers bench.py reports under "comparator");
* config 3: ogbn-products SAGE (mean values), k=32: SpGEMM + SSpMM through the autograd
  surface (maxk_kernels.maxk_aggregate forward + backward, top-k and MaxK scatter included)
  and the two plan kernels alone;
* config 4: ogbn-proteins GCN (symmetric normalisation), k in {8, 16, 32, 64}: forward and
  backward kernels with the algorithmic-byte roofline fraction (bench.py's formulas).

Graphs are the synthetic stand-ins of maxk_kernels.graphs (no datasets offline).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-gnn_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import maxk_kernels as mk  # noqa: E402
from maxk_kernels import graphs  # noqa: E402

HBM_PEAK_GBS = 8000.0


def timeit(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def kernel_times(ptr, idx, val, n, d, k, h, g):
    e = idx.numel()
    sp_data, sp_index = mk.maxk_forward(h, k, return_index=True)
    plan = mk.GraphPlan(ptr, idx, val, n, e, d, k)
    out = torch.empty((n, d), device=h.device)
    gs = torch.empty((n, k), device=h.device)
    tf = timeit(lambda: plan.forward(sp_data, sp_index, out))
    tb = timeit(lambda: plan.backward(g, sp_index, gs))
    fb = 4 * (n + 1) + 8 * e + 5 * k * n + 4 * d * n
    bb = 4 * (n + 1) + 8 * e + 4 * d * n + k * n + 4 * k * n
    return {"k": k, "fwd_ms": tf, "bwd_ms": tb, "edges_per_s": 2 * e / ((tf + tb) * 1e-3),
            "fwd_roofline_frac": fb / (tf * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "bwd_roofline_frac": bb / (tb * 1e-3) / 1e9 / HBM_PEAK_GBS}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    d = 256
    res = {}

    # config 2: Reddit forward vs rocSPARSE
    n, e = graphs.DATASETS["reddit"]
    ptr, idx = graphs.bench_csr("reddit", device=dev)
    val = graphs.sage_mean_values(ptr)
    h = graphs.features(n, d, seed=97, device=dev)
    sp_data, sp_index = mk.maxk_forward(h, 16, return_index=True)
    plan = mk.GraphPlan(ptr, idx, val, n, idx.numel(), d, 16)
    out = torch.empty((n, d), device=dev)
    tf = timeit(lambda: plan.forward(sp_data, sp_index, out))
    from maxk_kernels import baselines
    dense = torch.zeros((n, d), device=dev)
    dense.scatter_(1, sp_index.long(), sp_data)
    _, t_rs = baselines.spmm_rocsparse(ptr, idx, val, dense, times=10, alg="csr_merge_path")
    res["reddit_fwd_k16"] = {"spgemm_fwd_ms": tf, "rocsparse_spmm_ms": t_rs,
                             "speedup": t_rs / tf, "edges": idx.numel()}
    print(json.dumps(res["reddit_fwd_k16"]), flush=True)
    del ptr, idx, val, h, sp_data, sp_index, plan, out, dense
    torch.cuda.empty_cache()

    # config 3: ogbn-products SAGE, k = 32, autograd path and kernels
    n, e = graphs.DATASETS["ogbn-products"]
    ptr, idx = graphs.bench_csr("ogbn-products", device=dev)
    val = graphs.sage_mean_values(ptr)
    h = graphs.features(n, d, seed=97, device=dev)
    g = graphs.features(n, d, seed=98, device=dev)
    graph = mk.CSRGraph(ptr, idx, val)
    x = h.clone().requires_grad_(True)

    def step():
        y = mk.maxk_aggregate(x, graph, 32)
        y.backward(g)

    t_step = timeit(step, reps=10)
    kt = kernel_times(ptr, idx, val, n, d, 32, h, g)
    res["products_sage_k32"] = dict(kt, autograd_step_ms=t_step, edges=idx.numel(),
                                    autograd_edges_per_s=2 * idx.numel() / (t_step * 1e-3))
    print(json.dumps(res["products_sage_k32"]), flush=True)
    del ptr, idx, val, h, g, graph, x
    torch.cuda.empty_cache()

    # config 4: ogbn-proteins GCN, k sweep
    n, e = graphs.DATASETS["ogbn-proteins"]
    ptr, idx = graphs.bench_csr("ogbn-proteins", device=dev)
    val = graphs.gcn_values(ptr, idx)
    h = graphs.features(n, d, seed=97, device=dev)
    g = graphs.features(n, d, seed=98, device=dev)
    res["proteins_gcn"] = []
    for k in (8, 16, 32, 64):
        kt = kernel_times(ptr, idx, val, n, d, k, h, g)
        res["proteins_gcn"].append(kt)
        print(json.dumps(dict(kt, config="proteins_gcn")), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
