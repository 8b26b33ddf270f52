"""Small fixed workload for rocprofv3 --pmc passes (tooling): one dataset-shaped synthetic
graph (PMC_DATASET, default reddit; PMC_GRAPH uniform (default), community or shuffled as in
tools/locality_graphs.py), D=256, k=PMC_K, SAGE-mean or GCN values (PMC_KIND), 1 + 3 SpGEMM
forwards and 1 + 3 SSpMM backwards with the default (or PMC_OPTS) plan."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-gnn_amd"))
import torch  # noqa: E402

import maxk_kernels as mk  # noqa: E402
from maxk_kernels import graphs  # noqa: E402

k = int(os.environ.get("PMC_K", "16"))
ds = os.environ.get("PMC_DATASET", "reddit")
kind = os.environ.get("PMC_KIND", "sage")
dev = torch.device("cuda:0")
n, e = graphs.DATASETS[ds]
shape = os.environ.get("PMC_GRAPH", "uniform")
if shape == "uniform":
    ptr, idx = graphs.bench_csr(ds, device=dev)
else:
    ptr, idx = graphs.community_csr(n, e, shuffle=shape == "shuffled", device=dev)
val = graphs.sage_mean_values(ptr) if kind == "sage" else graphs.gcn_values(ptr, idx)
e = idx.numel()
h = graphs.features(n, 256, seed=97, device=dev)
g = graphs.features(n, 256, seed=98, device=dev)
sp_data, sp_index = mk.maxk_forward(h, k, return_index=True)
del h
opts = json.loads(os.environ.get("PMC_OPTS", "{}"))
plan = mk.GraphPlan(ptr, idx, val, n, e, 256, k, options=opts)
out = plan.forward(sp_data, sp_index)
grad = plan.backward(g, sp_index)
for _ in range(3):
    plan.forward(sp_data, sp_index, out)
for _ in range(3):
    plan.backward(g, sp_index, grad)
torch.cuda.synchronize()
# the kernel binary these counters belong to (tools/pmc_traffic.py stores it with the entry;
# bench.py drops a traffic figure whose binary differs from the one it loaded)
out_dir = os.environ.get("PMC_OUT")
if out_dir:
    with open(os.path.join(out_dir, "lib_sha256.txt"), "w") as f:
        f.write(mk._lib.lib_sha256() + "\n")
print("done", plan.info())
