"""Where a MaxK aggregation autograd step spends its time (tooling, round 5): Reddit-shaped bench
graph, D = 256, k = 16 (or --k), x [N, D] requiring grad; one step = maxk_aggregate(x, graph, k)
forward + backward with a given upstream gradient. Prints the step's device time (HIP events),
the host time per step (wall clock of the Python calls without synchronising, i.e. how long
the CPU takes to queue it), and the kernel times of its parts measured alone: top-k, SpGEMM,
SSpMM, MaxK scatter. Round 6: also the unfused composition (MaxKFunction -> SpGEMMFunction,
whose forward packs / scans the tables) in the same process, and the fused parts (top-k with
statistics in the plan's layout, forward given the statistics).

  python tools/autograd_step.py [--dataset reddit] [--k 16]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-gnn_amd"))
import torch  # noqa: E402

import maxk_kernels as mk  # noqa: E402
from maxk_kernels import graphs  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def host_time(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dataset", default="reddit")
    ap.add_argument("--k", type=int, default=16)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n, _ = graphs.DATASETS[args.dataset]
    ptr, idx = graphs.bench_csr(args.dataset, device=dev)
    graph = mk.CSRGraph(ptr, idx, graphs.sage_mean_values(ptr))
    d, k = 256, args.k
    x = graphs.features(n, d, seed=97, device=dev).requires_grad_(True)
    g = graphs.features(n, d, seed=98, device=dev)

    def step():  # x.grad accumulates across steps (no zero_grad), as in a loop without one
        y = mk.maxk_aggregate(x, graph, k)
        y.backward(g)

    def step_fresh():  # optimizer.zero_grad(set_to_none=True) before every step
        x.grad = None
        y = mk.maxk_aggregate(x, graph, k)
        y.backward(g)

    def step_unfused():  # round 5's composition: MaxKFunction -> SpGEMMFunction (the forward
        x.grad = None    # packs / scans the CBSR tables it is handed)
        sd, si = mk.maxk(x, k)
        y = mk.spgemm(sd, si, graph, d)
        y.backward(g)

    t_step = timeit(step)
    t_fresh = timeit(step_fresh)
    t_unfused = timeit(step_unfused)
    t_fresh2 = timeit(step_fresh)   # again, after the unfused variant (order effects)
    t_host = host_time(step_fresh)
    plan = graph.plan(d, k)
    sp_data, sp_index = mk.maxk_forward(x.detach(), k, return_index=True)
    out = torch.empty(n, d, device=dev)
    gsp = torch.empty(n, k, device=dev)
    rd, ri = plan.new_cbsr()
    st = torch.empty(2, dtype=torch.int32, device=dev)
    mk.maxk_forward(x.detach(), k, return_index=True, out=(rd, ri), stats=st)
    fused = {
        "topk_stats_layout_ms": timeit(lambda: mk.maxk_forward(x.detach(), k, return_index=True,
                                                                out=(rd, ri), stats=st)),
        "spgemm_fwd_given_stats_ms": timeit(lambda: plan.forward(rd, ri, out,
                                                                 stats=st.view(1, 2))),
    }
    parts = {
        "topk_ms": timeit(lambda: mk.maxk_forward(x.detach(), k, return_index=True)),
        "spgemm_fwd_ms": timeit(lambda: plan.forward(sp_data, sp_index, out)),
        "sspmm_bwd_ms": timeit(lambda: plan.backward(g, sp_index, gsp)),
        "maxk_scatter_ms": timeit(lambda: mk.maxk_backward(gsp, sp_index, d)),
    }
    print(json.dumps({"dataset": args.dataset, "k": k, "fwd_layout": plan.info()["fwd_layout"],
                      "step_ms": t_step, "step_ms_grad_none": t_fresh,
                      "step_ms_grad_none_again": t_fresh2, "step_ms_unfused": t_unfused,
                      "host_ms_per_step": t_host, "fused_parts": fused,
                      "parts": parts, "parts_sum_ms": sum(parts.values())}), flush=True)


if __name__ == "__main__":
    main()
