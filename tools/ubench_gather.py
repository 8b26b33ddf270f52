"""Drives tools/ubench_gather.hip (tooling). Run on the GPU box."""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, "libubench_gather.so"))
lib.ubench_gather.restype = ctypes.c_float
lib.ubench_gather.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 5 + [ctypes.c_int] * 4
dev = torch.device("cuda:0")
N, K = 232_965, 16
EPW = 8192
NWG = 115_000_000 // EPW
g = torch.Generator(device=dev).manual_seed(0)
idx = torch.randint(0, N, (NWG * EPW,), device=dev, generator=g, dtype=torch.int32)
# sort each 16-edge group's columns like CSR rows (ascending within a row)
data = torch.randn(N, K, device=dev, generator=g)
sel = torch.randint(0, 256, (N, K), device=dev, generator=g, dtype=torch.uint8)
packed = torch.zeros(N, 128, dtype=torch.uint8, device=dev)
out = torch.empty(NWG * 256, device=dev)
names = ["separate 64B+16B", "packed 128B", "packed 80B", "separate, window", "packed128, window",
         "values only"]
for v, w in [(1, 0), (4, -4096), (4, -16384), (4, -32768), (4, -65536), (3, -16384), (0, 0)]:
    ms = lib.ubench_gather(v, idx.data_ptr(), data.data_ptr(), sel.data_ptr(), packed.data_ptr(),
                           out.data_ptr(), NWG, EPW, max(w, 1), 5)
    e = NWG * EPW
    print(f"{v} {names[v]:20s} window={w:7d} {ms:7.3f} ms {e / ms / 1e6:7.2f} Gedges/s", flush=True)
