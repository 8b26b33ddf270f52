"""Drives tools/probe_topk2.hip (tooling, round 5): exact top-k variants on the Reddit and
ogbn-products feature matrices (N(0,1), seed 97, D = 256), device time per call and whether
the output equals the library's bit for bit. Build first (see the .hip header), then

  python tools/probe_topk2.py [out.jsonl]
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-gnn_amd"))

import torch  # noqa: E402

import maxk_kernels as mk  # noqa: E402
from maxk_kernels import graphs  # noqa: E402

lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libprobe_topk2.so"))
lib.probe_topk2.restype = ctypes.c_float
P = ctypes.c_void_p
lib.probe_topk2.argtypes = [ctypes.c_int] * 4 + [P] * 4 + [ctypes.c_int] * 3
out = open(sys.argv[1], "w") if len(sys.argv) > 1 else None
dev = torch.device("cuda:0")
CASES = [(0, 4, 1, 1, "library")] + \
        [(5, r, p, 1, f"dual R={r} P={p}") for r, p in ((2, 2), (4, 4), (4, 2), (8, 4), (8, 8))] + \
        [(4, r, p, 1, f"lean R={r} P={p}") for r, p in ((4, 4), (8, 8))] + \
        [(1, r, p, 1, f"pipelined R={r} P={p}") for r, p in ((4, 4), (8, 4), (2, 2))]
for name in ("reddit", "ogbn-products"):
    n, _ = graphs.DATASETS[name]
    h = graphs.features(n, 256, seed=97, device=dev)
    sink = torch.zeros(n, dtype=torch.int32, device=dev)
    for k in (8, 16, 32, 64):
        ref_d, ref_i = mk.maxk_forward(h, k, mode="exact", return_index=True)
        for var, r, p, rep, label in CASES:
            d = torch.zeros(n, k, device=dev)
            i = torch.zeros(n, k, dtype=torch.uint8, device=dev)
            ms = lib.probe_topk2(var, r, p, rep, P(h.data_ptr()), P(d.data_ptr()),
                                 P(i.data_ptr()), P(sink.data_ptr()), n, k, 20)
            torch.cuda.synchronize()
            ok = None if var == 2 else bool(torch.equal(d, ref_d) and torch.equal(i, ref_i))
            rec = {"dataset": name, "k": k, "variant": label, "ms": round(ms, 4),
                   "GBps": round((n * 256 * 4 + 5 * n * k) / ms / 1e6), "bit_exact": ok}
            print(json.dumps(rec), flush=True)
            if out:
                out.write(json.dumps(rec) + "\n")
    del h, sink
