"""Drives tools/ubench_lds.hip (tooling): times the forward inner loop's LDS-update variants
on Reddit-sized random gathers. Run on the GPU box: python tools/ubench_lds.py"""
import ctypes
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libubench_lds.so")
if not os.path.exists(SO):
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC",
                    os.path.join(HERE, "ubench_lds.hip"), "-o", SO], check=True)
lib = ctypes.CDLL(SO)
lib.ubench_run.restype = ctypes.c_float
lib.ubench_run.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int] * 3

N, K = 232_965, 16
EDGES_PER_WG = 8192
NWG = 115_000_000 // EDGES_PER_WG
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
idx = torch.randint(0, N, (NWG * EDGES_PER_WG,), device=dev, generator=g, dtype=torch.int32)
sp_data = torch.randn(N, K, device=dev, generator=g)
sp_index = torch.randint(0, 256, (N, K), device=dev, generator=g, dtype=torch.uint8)
out = torch.empty(NWG * 16 * 256, device=dev)
names = {0: "ds_add_f32 (product)", 1: "ds_read+ds_write RMW", 2: "no LDS update",
         3: "ds_add_f32 only (no gathers)", 4: "ds_add_u32", 5: "ds_add_f32 conflict-free, no gathers"}
for v in (0, 1, 2, 3, 4, 5):
    ms = lib.ubench_run(v, idx.data_ptr(), sp_data.data_ptr(), sp_index.data_ptr(),
                        out.data_ptr(), NWG, EDGES_PER_WG, 5)
    e = NWG * EDGES_PER_WG
    print(f"variant {v} {names[v]:38s} {ms:8.3f} ms  {e / ms / 1e6:8.2f} Gedges/s", flush=True)
sys.exit(0)
