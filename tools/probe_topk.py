"""Drives tools/probe_topk.hip (tooling): exact top-k time split into load / selection / emit,
and the emit staged through LDS, for rows per wave R in {1, 2, 4, 8}; modes 3 and 4 are checked
bit-exact against the product kernel. Build here, run on the GPU box:

  hipcc -O3 --offload-arch=gfx950 -shared -fPIC -Iinclude tools/probe_topk.hip -o tools/libprobe_topk.so
  python tools/probe_topk.py
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

lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libprobe_topk.so"))
lib.probe_topk.restype = ctypes.c_float
lib.probe_topk.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
MODES = {0: "load only", 1: "load + emit", 2: "select, no emit", 3: "product (select + emit)",
         4: "select + LDS-staged emit", 5: "rows batched per phase + LDS emit",
         6: "persistent 8 WG/CU, prefetch next rows", 7: "persistent 4 WG/CU, prefetch next rows"}
dev = torch.device("cuda:0")
for name in ("reddit", "ogbn-products"):
    n, _ = graphs.DATASETS[name]
    h = graphs.features(n, 256, seed=97, device=dev)
    for k in (16, 32):
        ref_d, ref_i = mk.maxk_forward(h, k, mode="exact", return_index=True)
        out = (torch.empty_like(ref_d), torch.empty_like(ref_i))
        for _ in range(3):
            mk.maxk_forward(h, k, out=out)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            mk.maxk_forward(h, k, out=out)
        b.record()
        b.synchronize()
        ms = a.elapsed_time(b) / 20
        print(json.dumps({"dataset": name, "k": k, "R": None, "mode": "product library",
                          "ms": round(ms, 4), "GBps": round(n * 256 * 4 / ms / 1e6)}), flush=True)
        for R in (1, 2, 4, 8):
            for mode in (MODES if len(sys.argv) < 2 else [int(m) for m in sys.argv[1].split(',')]):
                d = torch.zeros(n, k, device=dev)
                i = torch.zeros(n, k, dtype=torch.uint8, device=dev)
                ms = lib.probe_topk(mode, R, h.data_ptr(), d.data_ptr(), i.data_ptr(), n, k, 20)
                torch.cuda.synchronize()
                ok = None
                if mode >= 3:
                    ok = bool(torch.equal(d, ref_d) and torch.equal(i, ref_i))
                print(json.dumps({"dataset": name, "k": k, "R": R, "mode": MODES[mode],
                                  "ms": round(ms, 4), "GBps": round(n * 256 * 4 / ms / 1e6),
                                  "bit_exact": ok}), flush=True)
    del h
