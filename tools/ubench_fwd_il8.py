"""Drives tools/ubench_fwd_il8.hip (tooling): the 8-lanes-per-edge atomic-free SpGEMM forward
prototype (one dwordx3 gather per lane: 2 values + 2 selectors) on the Reddit-shaped graph at
k=16, checked against the product forward, by LDS mode, cv load form and column window.
Run on the GPU box: python tools/ubench_fwd_il8.py [--windows 0,8192]"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "spgemm-gnn_amd"))
sys.path.insert(0, HERE)
import torch  # noqa: E402

import maxk_kernels as mk  # noqa: E402
from maxk_kernels import graphs  # noqa: E402
from ubench_fwd_il import schedule  # noqa: E402

SO = os.path.join(HERE, "libubench_fwd_il8.so")
if not os.path.exists(SO):
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC",
                    os.path.join(HERE, "ubench_fwd_il8.hip"), "-o", SO], check=True)
lib = ctypes.CDLL(SO)
lib.ubench_fwd_il8.restype = ctypes.c_float
lib.ubench_fwd_il8.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                               ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_int]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", default="0,8192")
    ap.add_argument("--cap", type=int, default=4096)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n, e = graphs.DATASETS["reddit"]
    ptr, idx0 = graphs.synthetic_csr(n, e, device=dev)
    val = graphs.sage_mean_values(ptr)
    h = graphs.features(n, 256, seed=97, device=dev)
    sd, si = mk.maxk_forward(h, 16, return_index=True)
    # lane q: {x[2q], x[2q+1], sel[2q] | sel[2q+1] << 8} at q*12
    rec = torch.zeros(n, 32, dtype=torch.int32, device=dev)
    xi = sd.view(torch.int32).view(n, 8, 2)
    s2 = si.view(n, 8, 2).to(torch.int32)
    r3 = rec[:, :24].view(n, 8, 3)
    r3[:, :, 0] = xi[:, :, 0]
    r3[:, :, 1] = xi[:, :, 1]
    r3[:, :, 2] = s2[:, :, 0] | (s2[:, :, 1] << 8)
    rec = rec.contiguous()
    # 16-B lanes: {x[2q], x[2q+1], sel pair, 0} at q*16
    rec16 = torch.zeros(n, 8, 4, dtype=torch.int32, device=dev)
    rec16[:, :, :3] = r3
    rec16 = rec16.contiguous()
    for w in [int(x) for x in args.windows.split(",")]:
        idx = idx0 if w == 0 else (idx0 % w)
        if w:
            rows = torch.repeat_interleave(torch.arange(n, device=dev), (ptr[1:] - ptr[:-1]).long())
            key = rows * n + idx.long()
            idx = (torch.sort(key).values - rows * n).to(torch.int32)
        plan = mk.GraphPlan(ptr, idx, val, n, e, 256, 16)
        ref = plan.forward(sd, si)
        tref = None
        grp, ngrp, cvw, zrows, total = schedule(ptr, idx, val, args.cap, SLOTS=8)
        out = torch.empty(n, 256, device=dev)
        for nw, cw, r16 in [(1, 0, 0), (1, 0, 1), (1, 1, 1), (4, 0, 1), (4, 1, 1)]:
            rr = rec16 if r16 else rec
            if True:
                for mode in (0, 1, 2):
                    out.zero_()
                    lib.ubench_fwd_il8(mode, nw, cw, r16, grp.data_ptr(), ngrp, cvw.data_ptr(),
                                       rr.data_ptr(), out.data_ptr(), 0)
                    torch.cuda.synchronize()
                    err = float(((out - ref).abs() / (ref.abs() + 1e-3)).max()) if mode < 2 else None
                    ms = lib.ubench_fwd_il8(mode, nw, cw, r16, grp.data_ptr(), ngrp, cvw.data_ptr(),
                                            rr.data_ptr(), out.data_ptr(), 20)
                    print(json.dumps({"window": w, "nw": nw, "cv_wide": cw, "rec16": r16,
                                      "mode": ["rmw_f64", "atomic_f64", "no_lds"][mode],
                                      "ms": round(ms, 4), "slots_per_edge": round(total / e, 4),
                                      "max_rel_dev": err}), flush=True)
        del plan


if __name__ == "__main__":
    main()
