"""Bound model of the column-block backward (sspmm_bwd4_kernel) on the Reddit-shaped bench
graph (tooling): how many distinct grad_out lines each gather instruction
touches, from a host replay of the kernel's instruction composition, priced with the
per-line costs measured by tools/ubench_vec.hip (profiles/r03/ubench_vec.jsonl) and the L1 /
L2 hit rates of the PMC passes of tools/pmc_model.sh.

Replay: edges sorted by (column block, row) as the plan sorts them (identity column order,
ascending rows); a gather instruction covers EPS = 64 / L consecutive edges of a slot group's
stream, lane q of an edge gathers slot g * ns + q + L * i in instruction i (i < F), padding
slots (>= k) select feature 0. A line is (row, feature / 32): a grad_out row of D = 256 f32 is
8 lines of 128 B. A random sample of instruction groups is replayed (the mean is what the
model uses).

Price per gather instruction and CU (ubench_vec, 4-B lanes): max(4 ns, n1 * 0.42 + n2 * 0.95
+ n3 * 3.9) with n1 L1-hitting lines, n2 L1-missing L2 hits, n3 L2 misses (Infinity Cache /
HBM), split with the measured TCP_TCC_READ_REQ per gather instruction and TCC hit rate.

  python tools/bwd_model.py --k 16 --block-cols 1821 --groups 1 --pmc gpurun_out/pmc_model_reddit_k16
"""
import argparse
import ast
import csv
import glob
import json
import os
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-gnn_amd"))
import torch  # noqa: E402

from maxk_kernels import graphs  # noqa: E402

CUS = 256
NS_FLOOR, NS_L1, NS_L2, NS_MALL = 4.0, 0.42, 0.95, 3.9  # profiles/r03/ubench_vec.jsonl


def pmc_means(root, name="sspmm_bwd4"):
    """Mean counter value per dispatch and mean duration (ms) of the kernels matching name."""
    vals = defaultdict(list)
    durs = []
    for f in glob.glob(os.path.join(root, "pass*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if name in r.get("Kernel_Name", ""):
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in glob.glob(os.path.join(root, "pass*", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if name in r.get("Kernel_Name", ""):
                durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    out = {c: sum(v) / len(v) for c, v in vals.items()}
    if durs:
        out["ms"] = sorted(durs)[len(durs) // 2]
    return out


def plan_info(root):
    """The plan.info() line tools/pmc_driver.py printed (first pass log)."""
    for f in sorted(glob.glob(os.path.join(root, "pass*.log"))):
        for line in open(f):
            if line.startswith("done "):
                return ast.literal_eval(line[5:])
    return None


def replay(k, C, S, F, samples, seed=5):
    n, e = graphs.DATASETS["reddit"]
    ptr, idx = graphs.bench_csr("reddit")
    e = idx.numel()
    h = graphs.features(n, 256, seed=97)
    sel = torch.sort(torch.topk(h, k, dim=1).indices, dim=1).values.to(torch.int16)
    del h
    kp = -(-k // (F * S)) * F * S
    if kp > k:
        sel = torch.cat([sel, torch.zeros((n, kp - k), dtype=torch.int16)], 1)
    deg = (ptr[1:] - ptr[:-1]).long()
    rows = torch.repeat_interleave(torch.arange(n), deg)
    key = (idx.long() // C) * n + rows
    key, order = torch.sort(key, stable=True)
    pairs = int((key[1:] != key[:-1]).sum()) + 1
    del key
    ns = kp // S
    L = ns // F
    eps = 64 // L
    gen = torch.Generator().manual_seed(seed)
    starts = torch.randint(0, e // eps, (samples,), generator=gen) * eps
    edges = order[starts[:, None] + torch.arange(eps)]          # [samples, eps]
    r = rows[edges].numpy().astype(np.int64)
    c = idx.long()[edges]
    lines = []
    for g in range(S):
        for i in range(F):
            slots = g * ns + torch.arange(L) + L * i
            f = sel[c][:, :, slots].numpy().astype(np.int64)    # [samples, eps, L]
            ln = (r[:, :, None] * 8 + f // 32).reshape(samples, -1)
            ln.sort(axis=1)
            lines.append((np.diff(ln, axis=1) != 0).sum(axis=1) + 1)
    lines = np.concatenate(lines)
    return {"k": k, "kp": kp, "C": C, "S": S, "F": F, "L": L, "eps": eps, "edges": e,
            "pairs": pairs * S, "edges_per_pair": e / pairs,
            "gather_instr": e * kp // 64, "lines_per_instr": float(lines.mean()),
            "lines_per_instr_p10_p90": [float(np.percentile(lines, 10)),
                                        float(np.percentile(lines, 90))]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, required=True)
    ap.add_argument("--block-cols", type=int, default=0, help="C (default: from the PMC log)")
    ap.add_argument("--groups", type=int, default=0, help="S slot groups (default: 1 at k<32, else 2)")
    ap.add_argument("--fpl", type=int, default=4, help="F slots per lane")
    ap.add_argument("--samples", type=int, default=200000)
    ap.add_argument("--pmc", default="", help="gpurun_out/pmc_model_reddit_k<k>")
    a = ap.parse_args()
    info = plan_info(a.pmc) if a.pmc else None
    C = a.block_cols or (info or {}).get("bwd_block_cols")
    S = a.groups or (1 if a.k < 32 else 2)
    m = replay(a.k, C, S, a.fpl, a.samples)
    if a.pmc:
        p = pmc_means(a.pmc)
        m["pmc"] = {c: p[c] for c in sorted(p)}
        if "TCP_TCC_READ_REQ_sum" in p and "TCC_HIT_sum" in p:
            touches = m["gather_instr"] * m["lines_per_instr"]
            miss1 = min(1.0, p["TCP_TCC_READ_REQ_sum"] / touches)
            h2 = p["TCC_HIT_sum"] / max(1.0, p["TCC_HIT_sum"] + p["TCC_MISS_sum"])
            n = m["lines_per_instr"]
            per = max(NS_FLOOR, n * ((1 - miss1) * NS_L1 + miss1 * (h2 * NS_L2 + (1 - h2) * NS_MALL)))
            m["l1_miss_frac"] = miss1
            m["l2_hit"] = h2
            m["ns_per_gather_instr_pred"] = per
            m["pred_ms"] = m["gather_instr"] / CUS * per * 1e-6
            if "ms" in p:
                m["measured_ms"] = p["ms"]
                m["measured_over_pred"] = p["ms"] / m["pred_ms"]
                m["ns_per_gather_instr_measured"] = p["ms"] * 1e6 * CUS / m["gather_instr"]
    print(json.dumps(m), flush=True)


if __name__ == "__main__":
    main()
