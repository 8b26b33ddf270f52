import os, sys
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, os.path.join(ROOT, "spgemm-gnn_amd"))
import torch
import maxk_kernels as mk
from maxk_kernels import graphs
dev = torch.device("cuda:0")
n, e = graphs.DATASETS["reddit"]
ptr, idx = graphs.synthetic_csr(n, e, device=dev)
val = graphs.sage_mean_values(ptr)
h = graphs.features(n, 256, seed=97, device=dev)
sd, si = mk.maxk_forward(h, 16, return_index=True)
plan = mk.GraphPlan(ptr, idx, val, n, e, 256, 16)
st = mk.cbsr_stats(sd, si)
out = plan.forward(sd, si)
for _ in range(10):
    plan.forward(sd, si, out)
for _ in range(10):
    plan.forward(sd, si, out, stats=st)
torch.cuda.synchronize()
print("ok", st.cpu())
