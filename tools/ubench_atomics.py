"""Drives tools/ubench_atomics.hip (tooling). Run on the GPU box."""
import ctypes
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "spgemm-gnn_amd"))
SO = os.path.join(HERE, "libubench_atomics.so")
lib = ctypes.CDLL(SO)
lib.ubench_atomics.restype = ctypes.c_float
lib.ubench_atomics.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                               ctypes.c_int, ctypes.c_int]
lib.ubench_bwd.restype = ctypes.c_float
lib.ubench_bwd.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 6 + [ctypes.c_int] * 3
dev = torch.device("cuda:0")
NWG = 4096
table = torch.zeros(232_965 * 16, device=dev)
out = torch.empty(NWG * 256, device=dev)
adds = NWG * 256 * 256 * 4
names = ["ds_add_f32", "ds_add_u32", "ds_add_u64", "ds_add_f64", "ds RMW (racy)",
         "global f32 atomic agent", "global f32 atomic workgroup", "global store", "LDS f32 CAS add"]
for v in ():
    ms = lib.ubench_atomics(v, table.data_ptr(), table.numel(), out.data_ptr(), NWG, 3)
    print(f"{v} {names[v]:30s} {ms:8.3f} ms  {adds / ms / 1e6:9.2f} G adds/s", flush=True)

from maxk_kernels import graphs  # noqa: E402
N, E = graphs.DATASETS["reddit"]
ptr, idx = graphs.synthetic_csr(N, E, device=dev)
val = graphs.sage_mean_values(ptr)
rows = torch.repeat_interleave(torch.arange(N, device=dev), (ptr[1:] - ptr[:-1]).long())
G = torch.randn(N, 256, device=dev)
sp_index = torch.sort(torch.randint(0, 256, (N, 16), device=dev, dtype=torch.int32), 1).values.to(torch.uint8)
for C in (2400,):
    key = (idx.long() // C) * N + rows
    order = torch.argsort(key)
    erow, ecol, ev = rows[order].int().contiguous(), idx.long()[order].int().contiguous(), val[order].contiguous()
    nb = (N + C - 1) // C
    bounds = torch.searchsorted((idx.long() // C)[order].contiguous(), torch.arange(nb + 1, device=dev))
    tasks = []
    b = bounds.cpu().tolist()
    nch = max(1, 1024 // nb)
    for blk in range(nb):
        for i in range(nch):
            e0 = b[blk] + (b[blk + 1] - b[blk]) * i // nch
            e1 = b[blk] + (b[blk + 1] - b[blk]) * (i + 1) // nch
            tasks.append([blk * C, min(C, N - blk * C), e0, e1])
    tasks_t = torch.tensor(tasks, dtype=torch.int32, device=dev).contiguous()
    grad = torch.empty(N * 16, device=dev)
    for v, nm in [(3, "f32 CAS"), (5, "CAS, hot G"), (6, "CAS, no G"), (1, "racy RMW")]:
        lds = C * 16 * 4 * (2 if v == 4 else 1)
        if lds > 160 * 1024:
            continue
        ms = lib.ubench_bwd(v, tasks_t.data_ptr(), len(tasks), erow.data_ptr(), ecol.data_ptr(),
                            ev.data_ptr(), G.data_ptr(), sp_index.data_ptr(), grad.data_ptr(), 256,
                            lds, 3)
        print(f"bwd C={C} tasks={len(tasks)} {nm:12s} {ms:8.3f} ms  {E / ms / 1e6:8.2f} Gedges/s", flush=True)
