"""Model of a 16-B-chunk backward gather against today's dword gather (tooling, round 6;
VERDICT r05 item 6: price the candidate with the TD fit and the LDS constants before any GPU
minute). Host replay on the Reddit-shaped bench graph, exact top-k selectors:

  today     lane q of an edge gathers slot g * ns + q + L * i (dword), E * kp / 64 gather
            instructions, lines per instruction from the plan's (block, row) order
            (tools/bwd_model.py's replay);
  chunk16   each (edge, slot group) gathers the DISTINCT 16-B chunks of grad_out[row] that hold
            its selected features (one dwordx4 lane per chunk), lanes packed perfectly across
            edges (a per-call prefix sum of the chunk counts would be needed); a lane then
            adds 1-4 slots.

Priced with DESIGN §4.3's texture-data fit (11.4 + 1.62 x lines cycles per gather instruction,
lane width not a term: tools/ubench_vec.hip measured 4-B and 16-B lanes alike) and §4.6's LDS
constants (today's update: selector word + ds_read_b128 + 2 ds_cmpst_rtn_b64 per wave-step of
4 gather instructions = 57 cycles at k = 64; a chunk lane's slots are not adjacent in the
lane-ordered accumulator, so each costs one CAS, executed as max-slots-per-lane masked passes).

  python tools/bwd_chunk_model.py [--k 64] [--samples 20000]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-gnn_amd"))
import torch  # noqa: E402

from maxk_kernels import graphs  # noqa: E402

TD0, TD1 = 11.4, 1.62       # TD cycles per gather instruction: TD0 + TD1 x distinct lines
LDS_STEP_TODAY = 57.0       # LDS cycles per wave-step of 4 gather instructions (k = 64)
LDS_CAS = 57.0 / 4.0        # one CAS-class LDS instruction (the step has ~4 of that weight)
LDS_ADD64 = 10.8            # one 64-lane ds_add_u64 (3,428 G lane-updates/s chip-wide, §4.1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--groups", type=int, default=2)
    ap.add_argument("--block-cols", type=int, default=911)
    ap.add_argument("--samples", type=int, default=20000)
    a = ap.parse_args()
    k, S, C = a.k, a.groups, a.block_cols
    n, _ = graphs.DATASETS["reddit"]
    ptr, idx = graphs.bench_csr("reddit")
    e = idx.numel()
    h = graphs.features(n, 256, seed=97)
    sel = torch.sort(torch.topk(h, k, dim=1).indices, dim=1).values.numpy().astype(np.int64)
    del h
    ns = k // S
    deg = (ptr[1:] - ptr[:-1]).long()
    rows = torch.repeat_interleave(torch.arange(n), deg).numpy()
    key = (idx.long() // C).numpy() * n + rows
    order = np.argsort(key, kind="stable")
    del key
    cols = idx.numpy()
    rs = np.random.RandomState(5)
    res = {"k": k, "S": S, "C": C, "edges": e}
    for g in range(S):
        f = sel[:, g * ns:(g + 1) * ns]                       # [n, ns] this group's features
        ch = f // 4                                           # their 16-B chunks
        distinct = 1 + (np.diff(ch, axis=1) != 0).sum(axis=1)  # per column (sorted features)
        per_lane_max = np.zeros(n, np.int64)                  # most slots one chunk carries
        for c0 in range(0, n, 50000):
            blk = ch[c0:c0 + 50000]
            run = np.ones_like(blk)
            for j in range(1, ns):
                same = blk[:, j] == blk[:, j - 1]
                run[:, j] = np.where(same, run[:, j - 1] + 1, 1)
            per_lane_max[c0:c0 + 50000] = run.max(axis=1)
        # windows of consecutive edges in the plan order, expanded to (row, chunk) lanes
        lines_t, lines_c, passes = [], [], []
        L = ns // 4
        eps = 64 // L
        for s0 in rs.randint(0, e - 256, a.samples):
            ed = order[s0:s0 + 64]
            r, c = rows[ed], cols[ed]
            # today: eps edges per instruction, lane q slot q + L * i
            for i in range(4):
                fe = f[c[:eps]][:, np.arange(L) + L * i]
                lines_t.append(len(np.unique(r[:eps, None] * 8 + fe // 32)))
            # chunk16: the edges' distinct chunks, first 64 lanes
            lanes_r, lanes_ch, lanes_n = [], [], []
            for rr, cc in zip(r, c):
                u, cnt = np.unique(ch[cc], return_counts=True)
                lanes_r.extend([rr] * len(u))
                lanes_ch.extend(u)
                lanes_n.extend(cnt)
                if len(lanes_r) >= 64:
                    break
            lr, lc = np.array(lanes_r[:64]), np.array(lanes_ch[:64])
            lines_c.append(len(np.unique(lr * 8 + lc // 8)))
            passes.append(int(np.max(lanes_n[:64])))
        gi_t = e * ns / 64
        gi_c = float(distinct[cols].sum()) / 64
        lt, lc_, ps = float(np.mean(lines_t)), float(np.mean(lines_c)), float(np.mean(passes))
        td_t = gi_t * (TD0 + TD1 * lt)
        td_c = gi_c * (TD0 + TD1 * lc_)
        lds_t = gi_t / 4 * LDS_STEP_TODAY
        lds_c = gi_c * (ps + 1) * LDS_CAS          # masked CAS passes + the descriptor read
        lds_cf = gi_c * ps * LDS_ADD64             # fixed-point slots: one ds_add_u64 per pass
        res[f"group{g}"] = {
            "today": {"gather_instr": gi_t, "lines_per_instr": lt, "td_cycles": td_t,
                      "lds_cycles": lds_t},
            "chunk16": {"gather_instr": gi_c, "chunks_per_edge": float(distinct[cols].mean()),
                        "lines_per_instr": lc_, "cas_passes_per_instr": ps,
                        "td_cycles": td_c, "lds_cycles": lds_c,
                        "lds_cycles_fixed_point_adds": lds_cf},
        }
    tot = {d: {u: sum(res[f"group{g}"][d][u] for g in range(S)) for u in ("td_cycles", "lds_cycles")}
           for d in ("today", "chunk16")}
    for d in tot:
        tot[d]["bound_cycles"] = max(tot[d].values())
    res["total"] = tot
    res["predicted_change"] = tot["chunk16"]["bound_cycles"] / tot["today"]["bound_cycles"] - 1
    fx = sum(res[f"group{g}"]["chunk16"]["lds_cycles_fixed_point_adds"] for g in range(S))
    res["predicted_change_fixed_point_adds"] = (max(fx, tot["chunk16"]["td_cycles"]) /
                                                tot["today"]["bound_cycles"] - 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
