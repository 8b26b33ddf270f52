"""Drives tools/ubench_vec.hip (tooling): time per wave64 gather instruction and per record
("edge") by load width and lanes per record, for an L2-resident (1 MB) and a 32 MB table.
Run on the GPU box: python tools/ubench_vec.py [table MB list, default 1,32; 0.015625 = 16 KB
fits the 32 KB L1]"""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libubench_vec.so")
lib = ctypes.CDLL(SO)
lib.ubench_vec.restype = ctypes.c_float
lib.ubench_vec.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                           ctypes.c_int, ctypes.c_int]
dev = torch.device("cuda:0")
NWG = 256 * 8
ITERS = 512
PAT = [("16B x4 lanes (packed values)", 16, 4), ("4B x4 lanes at +64 (packed sel)", 4, 4),
       ("16B x6 lanes (lane chunks)", 16, 6), ("16B x8 lanes (128 B)", 16, 8),
       ("16B x5 lanes (80 B)", 16, 5), ("12B x8 lanes (96 B)", 12, 8),
       ("16B x2 lanes (32 B)", 16, 2), ("16B x1 lane", 16, 1), ("4B x1 lane", 4, 1),
       ("4B x16 lanes (64 B)", 4, 16), ("8B x4 lanes (32 B)", 8, 4), ("4B x4 lanes (16 B)", 4, 4)]
out = torch.empty(NWG * 256, dtype=torch.int32, device=dev)
for mb in [float(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,32").split(",")]:
    nrec = int(mb * 2**20) // 128
    table = torch.randint(0, 2**31 - 1, (nrec * 32,), dtype=torch.int32, device=dev)
    for p, (name, by, lpe) in enumerate(PAT):
        ms = lib.ubench_vec(p, table.data_ptr(), nrec, out.data_ptr(), NWG, 5)
        instr = NWG * 4 * ITERS
        ns_instr_cu = ms * 1e6 / (instr / 256)
        epi = 64 // lpe
        print(json.dumps({"table_MB": mb, "pattern": name, "bytes": by, "lanes_per_edge": lpe,
                          "edges_per_instr": epi, "ms": round(ms, 4),
                          "ns_per_instr_per_CU": round(ns_instr_cu, 2),
                          "ns_per_edge_per_CU": round(ns_instr_cu / epi, 3)}), flush=True)
sys.exit(0)
