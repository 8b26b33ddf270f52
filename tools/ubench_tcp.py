"""Drives tools/ubench_tcp.hip (tooling): time per wave64 dword-gather instruction by address
pattern, for an L2-resident (1 MB) and an Infinity-Cache-resident (64 MB) table. Run under
rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum --kernel-trace to get tag accesses per
instruction (kernel name tcp_kern<P>). Run on the GPU box: python tools/ubench_tcp.py"""
import ctypes
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libubench_tcp.so")
if not os.path.exists(SO):
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC",
                    os.path.join(HERE, "ubench_tcp.hip"), "-o", SO], check=True)
lib = ctypes.CDLL(SO)
lib.ubench_tcp.restype = ctypes.c_float
lib.ubench_tcp.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                           ctypes.c_int, ctypes.c_int]
dev = torch.device("cuda:0")
NWG = 256 * 8
ITERS = 512
names = ["same dword", "256 B contiguous", "16x(16 B in own line)", "16x(4 rnd in own 1KB row)",
         "4 edges/row, rnd in row quarter", "4x(16 rnd in own 1KB row)", "64 distinct lines",
         "16x(4 rnd in own row quarter)"]
out = torch.empty(NWG * 256, device=dev)
for rows in (1024, 65536):
    table = torch.randn(rows * 256, device=dev)
    for p in range(8):
        ms = lib.ubench_tcp(p, table.data_ptr(), rows, out.data_ptr(), NWG, 5)
        instr = NWG * 4 * ITERS
        ns_per_instr_cu = ms * 1e6 / (instr / 256)
        print(f"table {rows * 1024 / 2**20:5.0f} MB  P{p} {names[p]:34s} {ms:7.3f} ms "
              f"{ns_per_instr_cu:6.2f} ns/instr/CU", flush=True)
sys.exit(0)
