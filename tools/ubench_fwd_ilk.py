"""Drives tools/ubench_fwd_ilk.hip (tooling): the atomic-free interleaved SpGEMM forward at
k = 16/32/64 on the Reddit-shaped graph, against the product forward (same process), checked
against it. Variants: read-add-write vs ds_add_f64, clock-rotated sweeps (ticks per step).
  python tools/ubench_fwd_ilk.py [--k 32,64] [--tps 0,20,40]"""
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

SO = os.path.join(HERE, "libubench_fwd_ilk.so")
if not os.path.exists(SO):
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC",
                    os.path.join(HERE, "ubench_fwd_ilk.hip"), "-o", SO], check=True)
lib = ctypes.CDLL(SO)
lib.ubench_fwd_ilk.restype = ctypes.c_float
lib.ubench_fwd_ilk.argtypes = [ctypes.c_int] * 5 + [ctypes.c_void_p, ctypes.c_int] + \
    [ctypes.c_void_p] * 4 + [ctypes.c_int]


def schedule(ptr, idx, val, cap, slots):
    """Virtual rows (segments of <= cap edges) sorted by length, `slots` per group; the d
    edges of a slot in a group of T steps sit at steps floor(i * T / d) (spread evenly, so
    every slot is at the same column fraction at every step); other steps are padding."""
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
    ngrp = (nv + slots - 1) // slots
    padn = ngrp * slots - nv
    if padn:
        z = torch.zeros(padn, dtype=torch.long, device=dev)
        seg_row = torch.cat([seg_row, z - 1])
        seg_start = torch.cat([seg_start, z])
        seg_len = torch.cat([seg_len, z])
        split = torch.cat([split, torch.zeros(padn, dtype=torch.bool, device=dev)])
    steps = seg_len.view(ngrp, slots).max(1).values
    base = (torch.cumsum(steps, 0) - steps) * slots
    total = int(steps.sum()) * slots
    cvw = torch.zeros(total, 2, dtype=torch.int32, device=dev)
    cvw[:, 0] = -1
    v_of_e = torch.repeat_interleave(torch.arange(ngrp * slots, device=dev), seg_len)
    i = torch.arange(v_of_e.numel(), device=dev) - (torch.cumsum(seg_len, 0) - seg_len)[v_of_e]
    e = seg_start[v_of_e] + i
    T = steps[v_of_e // slots]
    t = (i * T) // seg_len[v_of_e]
    pos = base[v_of_e // slots] + t * slots + (v_of_e % slots)
    cvw[pos, 0] = idx.long()[e].to(torch.int32)
    cvw[pos, 1] = val[e].view(torch.int32)
    rows = seg_row.view(ngrp, slots).to(torch.int32)
    rows = torch.where(split.view(ngrp, slots) & (rows >= 0), rows | (-2**31), rows)
    grp = torch.zeros(ngrp, 2 + slots, dtype=torch.int32, device=dev)
    grp[:, 0] = base.to(torch.int32)
    grp[:, 1] = steps.to(torch.int32)
    grp[:, 2:] = rows
    zero_rows = torch.unique(seg_row[split & (seg_row >= 0)])
    return grp.contiguous(), ngrp, cvw.contiguous(), zero_rows, total


def timeit(fn, reps=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", default="32,64")
    ap.add_argument("--tps", default="0,20,40,80")
    ap.add_argument("--cap", type=int, default=4096)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n, e = graphs.DATASETS["reddit"]
    ptr, idx = graphs.synthetic_csr(n, e, device=dev)
    val = graphs.sage_mean_values(ptr)
    h = graphs.features(n, 256, seed=97, device=dev)
    out = torch.empty(n, 256, device=dev)
    for k in [int(x) for x in args.k.split(",")]:
        sd, si = mk.maxk_forward(h, k, return_index=True)
        plan = mk.GraphPlan(ptr, idx, val, n, e, 256, k)
        ref = plan.forward(sd, si)
        tprod = timeit(lambda: plan.forward(sd, si, ref))
        del plan
        slots = 64 // (k // 4)
        grp, ngrp, cvw, zrows, total = schedule(ptr, idx, val, args.cap, slots)
        print(json.dumps({"k": k, "product_ms": round(tprod, 4), "slots_per_edge": total / e}),
              flush=True)
        for tps in [int(x) for x in args.tps.split(",")]:
            for mode in (0, 1):
                for u16 in (0, 1):
                    out.zero_()
                    lib.ubench_fwd_ilk(k, mode, int(tps > 0), u16, max(tps, 1), grp.data_ptr(), ngrp,
                                       cvw.data_ptr(), sd.data_ptr(), si.data_ptr(), out.data_ptr(), 0)
                    torch.cuda.synchronize()
                    err = float(((out - ref).abs() / (ref.abs() + 1e-3)).max())
                    ms = lib.ubench_fwd_ilk(k, mode, int(tps > 0), u16, max(tps, 1), grp.data_ptr(),
                                            ngrp, cvw.data_ptr(), sd.data_ptr(), si.data_ptr(),
                                            out.data_ptr(), 10)
                    print(json.dumps({"k": k, "tps": tps, "mode": ["rmw_f64", "atomic_f64"][mode],
                                      "U": 16 if u16 else 8, "ms": round(ms, 4),
                                      "max_rel_dev": err}), flush=True)


if __name__ == "__main__":
    main()
