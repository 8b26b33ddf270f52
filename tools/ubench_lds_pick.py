"""Drives tools/ubench_lds_pick.hip (tooling, round 5): LDS cycles per wave-step of the current
backward update and of the LDS-staged candidate's picks and row staging, with real selector
words (sorted exact top-k of N(0,1) rows, the kernel's lane order). Cycles = device time x
2.26 GHz (the clock GRBM_GUI_ACTIVE gives under these kernels) / (8 waves x
iters) per CU. Output: one JSON line per (k, mode), also appended to argv[1] if given.

  python tools/ubench_lds_pick.py [out.jsonl]
"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libubench_lds_pick.so"))
lib.ubench_lds_pick.restype = ctypes.c_float
P = ctypes.c_void_p
lib.ubench_lds_pick.argtypes = [ctypes.c_int, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P,
                                ctypes.c_int, ctypes.c_int, ctypes.c_int, P, ctypes.c_int]
CLK = 2.26e9
dev = torch.device("cuda:0")
cus = torch.cuda.get_device_properties(0).multi_processor_count
out = open(sys.argv[1], "a") if len(sys.argv) > 1 else None
g = torch.Generator(device=dev)
g.manual_seed(5)
x = torch.randn(1024, 256, generator=g, device=dev)
gsrc = torch.randn(2048, 256, generator=g, device=dev)   # 2 MB: L2-resident rows
sink = torch.zeros(cus * 512, device=dev)
ITERS = 4096
# (k, slots per group ns, C): k = 16 one group of 16 slots; k = 64 two groups of 32
for k, ns, C in ((16, 16, 1024), (32, 16, 1024), (64, 32, 480)):
    L = ns // 4
    sel = torch.topk(x, k, dim=1).indices.sort(dim=1).values.to(torch.int64)[:, :ns]
    # lane-ordered words of group 0: lane q holds slots q, q + L, q + 2L, q + 3L
    sw = torch.zeros(1024, L, dtype=torch.int64, device=dev)
    for j in range(4):
        sw |= sel[:, j * L:(j + 1) * L] << (8 * j)
    sw = sw.to(torch.int32).contiguous()
    for mode, dma_every, label in ((0, 1, "picks (sel word + 4 ds_read_b32)"),
                                   (1, 1, "update (sel word + b128 + 2 cmpst_b64)"),
                                   (2, 1, "staging (global_load_lds_dwordx4, 1 KB)"),
                                   (3, 1, "picks + update + DMA every step"),
                                   (3, 4, "picks + update + DMA every 4 steps"),
                                   (4, 1, "staging via registers (dwordx4 + ds_write_b128)"),
                                   (5, 1, "picks + update + reg-staged row every step"),
                                   (5, 2, "picks + update + reg-staged row every 2 steps"),
                                   (5, 4, "picks + update + reg-staged row every 4 steps")):
        src = gsrc
        ms = lib.ubench_lds_pick(mode, P(sw.data_ptr()), L, C, dma_every, P(src.data_ptr()),
                                 src.shape[0], ITERS, cus, P(sink.data_ptr()), 10)
        torch.cuda.synchronize()
        cyc = ms * 1e-3 * CLK / (8 * ITERS) if ms > 0 else None
        rec = {"k": k, "slots_per_group": ns, "lanes_per_edge": L, "edges_per_step": 64 // L,
               "mode": label, "dma_every": dma_every, "ms": round(ms, 4),
               "cycles_per_wave_step": None if cyc is None else round(cyc, 2)}
        print(json.dumps(rec), flush=True)
        if out:
            out.write(json.dumps(rec) + "\n")
