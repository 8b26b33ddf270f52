"""MaxK top-k -> CBSR timing on the BASELINE shapes (tooling): exact and ref_compat modes,
device time per call (HIP events, mean of 20 after warm-up) and achieved HBM GB/s against
the N*D*4 read + 5*N*k write; with and without the fused statistics (maxk_topk_cbsr_ex).

  python tools/topk_time.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-gnn_amd"))

import torch  # noqa: E402

import maxk_kernels as mk  # noqa: E402
from maxk_kernels import graphs  # noqa: E402

dev = torch.device("cuda:0")
for name in ("reddit", "ogbn-products"):
    n, _ = graphs.DATASETS[name]
    h = graphs.features(n, 256, seed=97, device=dev)
    for k in (8, 16, 32, 64):
        st = torch.empty(2, dtype=torch.int32, device=dev)
        for mode, stats in (("exact", None), ("exact", st), ("ref_compat", None),
                            ("ref_compat", st)):
            fn = lambda: mk.maxk_forward(h, k, mode=mode, return_index=True, stats=stats)  # noqa: E731
            for _ in range(3):
                fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(20):
                fn()
            e.record()
            e.synchronize()
            ms = s.elapsed_time(e) / 20
            byts = n * 256 * 4 + 5 * n * k
            print(json.dumps({"dataset": name, "k": k, "mode": mode, "stats": stats is not None,
                              "ms": ms,
                              "GBps": byts / ms / 1e6}), flush=True)
    del h
