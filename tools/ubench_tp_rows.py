"""Drives tools/ubench_tp_rows.hip (tooling): the two-pass backward's row pass on an
ogbn-products-shaped problem (N = 2,449,029, E = 123,718,280, k = 32, D = 256, 4 rows per
wavefront), by variant; the product-writing variants are checked equal to variant 0.

  hipcc -O3 --offload-arch=gfx950 -shared -fPIC tools/ubench_tp_rows.hip -o tools/libubench_tp_rows.so
  python tools/ubench_tp_rows.py            # one JSON line per variant
"""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "spgemm-gnn_amd"))
from maxk_kernels import graphs  # noqa: E402

lib = ctypes.CDLL(os.path.join(HERE, "libubench_tp_rows.so"))
lib.ubench_tp_rows.restype = ctypes.c_float
lib.ubench_tp_rows.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 5 + [ctypes.c_int] * 3 + \
                              [ctypes.c_void_p, ctypes.c_int]
NAMES = {0: "product (nt stores)", 1: "plain stores", 2: "pipelined, nt stores",
         3: "pipelined, plain stores", 4: "probe: no stores", 5: "pipelined, sc1 stores"}

dev = torch.device("cuda:0")
n, e = graphs.DATASETS["ogbn-products"]
d, k, R = 256, 32, 4
ptr = graphs.synthetic_ptr(n, e, seed=97, device=dev)
idx = graphs.synthetic_rows(ptr, seed=97)
rows = torch.repeat_interleave(torch.arange(n, device=dev), (ptr[1:] - ptr[:-1]).long(),
                               output_size=e)
val = graphs.sage_mean_values(ptr, num_edges=e)
erec32 = torch.empty((e, 2), dtype=torch.int32, device=dev)
erec32[:, 0] = (idx.long() | ((rows % R) << 26)).to(torch.int32)
erec32[:, 1] = val.view(torch.int32)
del rows
G = graphs.features(n, d, seed=98, device=dev)
sel = torch.sort(torch.argsort(torch.rand(n, d, device=dev), dim=1)[:, :k], dim=1).values
sel = sel.to(torch.uint8).contiguous()
T = torch.empty((e, k), dtype=torch.float32, device=dev)
sink = torch.zeros(4, dtype=torch.int32, device=dev)
ref = None
for var in (0, 1, 2, 3, 5, 4):
    T.zero_()
    ms = lib.ubench_tp_rows(var, ptr.data_ptr(), erec32.data_ptr(), G.data_ptr(), sel.data_ptr(),
                            T.data_ptr(), n, d, k, sink.data_ptr(), 5)
    torch.cuda.synchronize()
    same = None
    if var != 4:
        h = torch.sum(T.view(torch.int32).view(-1)[::97].long()).item()
        ref = h if ref is None else ref
        same = h == ref
    print(json.dumps({"variant": var, "name": NAMES[var], "ms": round(ms, 4),
                      "write_TBps": None if var == 4 else round(e * k * 4 / (ms * 1e-3) / 1e12, 2),
                      "same_products": same}), flush=True)
