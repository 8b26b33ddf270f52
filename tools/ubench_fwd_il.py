"""Drives tools/ubench_fwd_il.hip (tooling): the atomic-free interleaved SpGEMM forward
prototype on the Reddit-shaped graph at k=16, checked against the product forward, by LDS
mode and column window (window W folds every column into [0, W): an L2-resident table).
Run on the GPU box: python tools/ubench_fwd_il.py [--windows 0,8192] [--cap 4096]"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "spgemm-gnn_amd"))
import torch  # noqa: E402

import maxk_kernels as mk  # noqa: E402
from maxk_kernels import graphs  # noqa: E402

SO = os.path.join(HERE, "libubench_fwd_il.so")
if not os.path.exists(SO):
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC",
                    os.path.join(HERE, "ubench_fwd_il.hip"), "-o", SO], check=True)
lib = ctypes.CDLL(SO)
lib.ubench_fwd_il.restype = ctypes.c_float
lib.ubench_fwd_il.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
SLOTS = 16


def schedule(ptr, idx, val, cap, SLOTS=SLOTS):
    """Virtual rows (row segments of <= cap edges), sorted by length, 16 per group; each group
    interleaves one edge of each of its rows per step."""
    dev = ptr.device
    n = ptr.numel() - 1
    deg = (ptr[1:] - ptr[:-1]).long()
    nseg = torch.clamp((deg + cap - 1) // cap, min=1)
    seg_row = torch.repeat_interleave(torch.arange(n, device=dev), nseg)
    first = torch.cumsum(nseg, 0) - nseg
    seg_k = torch.arange(seg_row.numel(), device=dev) - first[seg_row]
    seg_start = ptr[:-1].long()[seg_row] + seg_k * cap
    seg_len = torch.minimum(deg[seg_row] - seg_k * cap, torch.full_like(seg_k, cap)).clamp(min=0)
    split = nseg[seg_row] > 1
    order = torch.argsort(seg_len, descending=True, stable=True)
    seg_row, seg_start, seg_len, split = seg_row[order], seg_start[order], seg_len[order], split[order]
    nv = seg_row.numel()
    ngrp = (nv + SLOTS - 1) // SLOTS
    padn = ngrp * SLOTS - nv
    if padn:
        z = torch.zeros(padn, dtype=torch.long, device=dev)
        seg_row = torch.cat([seg_row, z - 1])
        seg_start = torch.cat([seg_start, z])
        seg_len = torch.cat([seg_len, z])
        split = torch.cat([split, torch.zeros(padn, dtype=torch.bool, device=dev)])
    steps = seg_len.view(ngrp, SLOTS).max(1).values
    base = (torch.cumsum(steps, 0) - steps) * SLOTS
    total = int(steps.sum()) * SLOTS
    cvw = torch.zeros(total, 2, dtype=torch.int32, device=dev)
    # every real edge of virtual row v: position base[g] + t*16 + j
    v_of_e = torch.repeat_interleave(torch.arange(ngrp * SLOTS, device=dev), seg_len)
    t = torch.arange(v_of_e.numel(), device=dev) - (torch.cumsum(seg_len, 0) - seg_len)[v_of_e]
    e = seg_start[v_of_e] + t
    pos = base[v_of_e // SLOTS] + t * SLOTS + (v_of_e % SLOTS)
    cvw[pos, 0] = idx.long()[e].to(torch.int32)
    cvw[pos, 1] = val[e].view(torch.int32)
    rows = seg_row.view(ngrp, SLOTS).to(torch.int32)
    rows = torch.where(split.view(ngrp, SLOTS) & (rows >= 0), rows | (-2**31), rows)
    grp = torch.zeros(ngrp, 4 + SLOTS, dtype=torch.int32, device=dev)
    grp[:, 0] = base.to(torch.int32)
    grp[:, 1] = steps.to(torch.int32)
    grp[:, 4:] = rows.to(torch.int32)
    zero_rows = torch.unique(seg_row[split & (seg_row >= 0)])
    return grp.contiguous(), ngrp, cvw.contiguous(), zero_rows, total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", default="0,8192")
    ap.add_argument("--cap", type=int, default=4096)
    ap.add_argument("--nw", default="4,1")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n, e = graphs.DATASETS["reddit"]
    ptr, idx0 = graphs.synthetic_csr(n, e, device=dev)
    val = graphs.sage_mean_values(ptr)
    h = graphs.features(n, 256, seed=97, device=dev)
    sd, si = mk.maxk_forward(h, 16, return_index=True)
    rec = torch.zeros(n, 128, dtype=torch.uint8, device=dev)
    rec[:, :64] = sd.view(torch.uint8).view(n, 64)
    rec[:, 64:80] = si
    for w in [int(x) for x in args.windows.split(",")]:
        idx = idx0 if w == 0 else (idx0 % w)
        if w:
            rows = torch.repeat_interleave(torch.arange(n, device=dev), (ptr[1:] - ptr[:-1]).long())
            key = rows * n + idx.long()
            idx = (torch.sort(key).values - rows * n).to(torch.int32)
        plan = mk.GraphPlan(ptr, idx, val, n, e, 256, 16)
        ref = plan.forward(sd, si)
        grp, ngrp, cvw, zrows, total = schedule(ptr, idx, val, args.cap)
        out = torch.empty(n, 256, device=dev)
        for nw, u16 in [(4, 0), (4, 1)]:
            for mode in (0, 1, 2, 3):
                out.zero_()
                lib.ubench_fwd_il(mode, nw, grp.data_ptr(), ngrp, cvw.data_ptr(), rec.data_ptr(),
                                  out.data_ptr(), 0, u16)
                torch.cuda.synchronize()
                err = float(((out - ref).abs() / (ref.abs() + 1e-3)).max()) if mode < 2 else None
                if mode == 2 and u16:
                    continue
                ms = lib.ubench_fwd_il(mode, nw, grp.data_ptr(), ngrp, cvw.data_ptr(),
                                       rec.data_ptr(), out.data_ptr(), 20, u16)
                print(json.dumps({"window": w, "nw": nw, "U": 16 if u16 else 8,
                                  "mode": ["rmw_f64", "atomic_f64", "no_lds", "no_lds_alloc0"][mode],
                                  "ms": round(ms, 4), "slots_per_edge": total / e,
                                  "max_rel_dev": err}), flush=True)
        del plan


if __name__ == "__main__":
    main()
