"""Host-side cost per call (tooling): ctypes launch path of GraphPlan.forward / backward and of
the autograd maxk_aggregate step on small graphs, against the GPU time of the same calls."""
import sys, time, json
sys.path.insert(0, "spgemm-gnn_amd")
import torch
import maxk_kernels as mk
from maxk_kernels import graphs
dev = torch.device("cuda:0")
for n, e in [(2000, 20000), (89250, 899756)]:
    ptr, idx = graphs.synthetic_csr(n, e, device=dev)
    val = graphs.sage_mean_values(ptr)
    h = graphs.features(n, 256, seed=1, device=dev)
    g = graphs.features(n, 256, seed=2, device=dev)
    sd, si = mk.maxk_forward(h, 16, return_index=True)
    plan = mk.GraphPlan(ptr, idx, val, n, idx.numel(), 256, 16)
    out = torch.empty((n, 256), device=dev); gs = torch.empty((n, 16), device=dev)
    for _ in range(20):
        plan.forward(sd, si, out); plan.backward(g, si, gs)
    torch.cuda.synchronize()
    reps = 500
    t0 = time.perf_counter()
    for _ in range(reps):
        plan.forward(sd, si, out)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    for _ in range(reps):
        plan.backward(g, si, gs)
    t3 = time.perf_counter()
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    s, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps): plan.forward(sd, si, out)
    en.record(); en.synchronize()
    gpu_f = s.elapsed_time(en) / reps
    # autograd path
    graph = mk.CSRGraph(ptr, idx, val)
    x = h.clone().requires_grad_(True)
    for _ in range(5):
        y = mk.maxk_aggregate(x, graph, 16); y.backward(g)
    torch.cuda.synchronize()
    t5 = time.perf_counter()
    for _ in range(100):
        y = mk.maxk_aggregate(x, graph, 16); y.backward(g)
    torch.cuda.synchronize()
    t6 = time.perf_counter()
    print(json.dumps({"n": n, "e": e, "fwd_host_us": (t1 - t0) / reps * 1e6, "fwd_wall_us": (t2 - t0) / reps * 1e6,
                      "bwd_host_us": (t3 - t2) / reps * 1e6, "fwd_gpu_us": gpu_f * 1e3,
                      "autograd_step_us": (t6 - t5) / 100 * 1e6}))
