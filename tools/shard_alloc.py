"""Which buffer's placement makes an 8-GPU rank's backward fast or slow (tooling, round 6;
VERDICT r05 item 3). One rank's ShardedAggregation (as tools/shard_time.py builds it). The
plan stays fixed; the backward is launched through the C ABI with each per-call buffer placed
at chosen byte offsets inside 2 MiB-aligned arenas (one buffer moved at a time, the others at
offset 0), and timed (HIP events, median of 3 rounds of 20):

  out   grad_sp [padded_rows, k] f32 (the C x k block stores at the end of every task)
  ws    the slab workspace (extra pieces of split blocks; read by the combine launch)
  gout  the rank's grad_out rows [n_local, D] f32 (gathered)
  sel   the gathered record table (selectors at the record stride)

Then the shard's plan (plan 0) and P fresh plans (new hipMallocs inside each plan), all per-call
buffers at offset 0, each timed twice in turn. Offset lines carry the buffers' virtual
addresses and their offsets within a 2 MiB fragment. MAXK_PLAN_MALLOC=contiguous makes the
plans allocate their streamed arrays physically contiguous (plan.hip plan_malloc).

  python tools/shard_alloc.py [--rank 3] [--world 8] [--k 16] [--offsets 0,4096,...]
                              [--plans 8] [--only out:0,out:1048576]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spgemm-gnn_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import maxk_kernels as mk  # noqa: E402
from maxk_kernels import graphs  # noqa: E402
from maxk_kernels._lib import check, lib  # noqa: E402
from maxk_kernels.dist import RowPartition, ShardedAggregation, record_views  # noqa: E402
from shard_time import timeit  # noqa: E402

FRAG = 2 << 20
P = ctypes.c_void_p


class Arena:
    """A buffer of `nbytes` placed at byte offset `off` from a 2 MiB-aligned address."""

    def __init__(self, nbytes, dev):
        self.raw = torch.empty(nbytes + 2 * FRAG, dtype=torch.uint8, device=dev)
        self.base = (-self.raw.data_ptr()) % FRAG
        self.nbytes = nbytes

    def at(self, off):
        a = self.base + off
        return self.raw[a:a + self.nbytes]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, default=3)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--offsets", default="0,256,4096,16384,65536,262144,524288,1048576,1572864")
    ap.add_argument("--plans", type=int, default=8)
    ap.add_argument("--only", default="", help="buf:off,... : time just these placements "
                    "(for PMC passes); plans are skipped")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cross", default="",
                    help="buf: time every plan (shard's + --plans fresh) at every --offsets "
                         "placement of that buffer, twice (a plan x offset matrix; out or ws "
                         "only: the placements of one arena overlap)")
    ap.add_argument("--plans-only", action="store_true",
                    help="skip the offset sweep: the shard's plan and --plans fresh plans, each "
                         "timed twice (MAXK_PLAN_MALLOC selects their allocation)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n, e = graphs.DATASETS["reddit"]
    ptr = graphs.synthetic_ptr(n, e, seed=97, device=dev)
    d, k = 256, args.k
    h = graphs.features(n, d, seed=97, device=dev)
    g = graphs.features(n, d, seed=98, device=dev)
    sd, si = mk.maxk_forward(h, k, return_index=True)
    del h
    part = RowPartition(ptr, args.world)
    q = args.rank
    a, b = part.rows(q)
    idx_q = graphs.synthetic_rows(ptr, seed=97, rows=(a, b))
    val_q = graphs.sage_mean_values(ptr[a:b + 1], num_edges=idx_q.numel())
    shard = ShardedAggregation(part, q, ptr, idx_q, val_q, d, k, local_edges=True)
    for r in range(args.world):
        pos = part.table_positions(r, dev)
        ra, rb = part.rows(r)
        shard.table_data[pos] = sd[ra:rb]
        shard.table_index[pos] = si[ra:rb]
    plan = shard.plan
    rec = shard.table_rec
    nloc, ncol = plan.num_rows, plan.num_cols
    wsb = plan.bwd_ws_bytes
    arenas = {"out": Arena(ncol * k * 4, dev), "ws": Arena(max(wsb, 256), dev),
              "gout": Arena(nloc * d * 4, dev), "sel": Arena(rec.numel(), dev)}
    gl = g[a:b].contiguous()
    stream = P(torch.cuda.current_stream().cuda_stream)
    pr, ix, vl = plan._refs

    def views(place):
        out = arenas["out"].at(place["out"]).view(torch.float32).view(ncol, k)
        ws = arenas["ws"].at(place["ws"])
        go = arenas["gout"].at(place["gout"]).view(torch.float32).view(nloc, d)
        rc = arenas["sel"].at(place["sel"]).view(rec.shape)
        return out, ws, go, rc

    def setup(place):
        out, ws, go, rc = views(place)
        go.copy_(gl)
        rc.copy_(rec)
        return out, ws, go, rc

    def launch(pl, out, ws, go, rc):
        ti = record_views(rc, k)[1]
        check(lib.maxk_sspmm_backward_tables(pl.handle, P(pr.data_ptr()), P(ix.data_ptr()),
                                             P(vl.data_ptr()), P(go.data_ptr()),
                                             P(ti.data_ptr()), ti.stride(0), P(out.data_ptr()),
                                             nloc, pl.num_edges, k, d, P(ws.data_ptr()), wsb,
                                             stream), "backward")

    def addrs(out, ws, go, rc):
        return {nm: {"va": hex(t.data_ptr()), "frag_off": t.data_ptr() % FRAG}
                for nm, t in (("out", out), ("ws", ws), ("gout", go), ("sel", rc))}

    zero = {"out": 0, "ws": 0, "gout": 0, "sel": 0}
    ref = setup(zero)
    launch(plan, *ref)
    torch.cuda.synchronize()
    want = ref[0].clone()
    if args.only:
        for spec in args.only.split(","):
            nm, off = spec.split(":")
            place = dict(zero, **{nm: int(off)})
            v = setup(place)
            ms = timeit(lambda: launch(plan, *v), reps=args.reps)
            print(json.dumps({"rank": q, "buf": nm, "off": int(off), "bwd_ms": ms}), flush=True)
        return
    if args.cross:
        plans = [plan] + [mk.GraphPlan(pr, ix, vl, nloc, plan.num_edges, d, k, num_cols=ncol)
                          for _ in range(args.plans)]
        offs = [int(x) for x in args.offsets.split(",")]
        views_at = {off: setup(dict(zero, **{args.cross: off})) for off in offs}
        for rnd in range(2):
            for i, p2 in enumerate(plans):
                row = [timeit(lambda: launch(p2, *views_at[off]), reps=args.reps) for off in offs]
                print(json.dumps({"rank": q, "buf": args.cross, "plan": i, "round": rnd,
                                  "offsets": offs, "bwd_ms": row}), flush=True)
        return
    for nm in (() if args.plans_only else ("out", "ws", "gout", "sel")):
        for off in [int(x) for x in args.offsets.split(",")]:
            place = dict(zero, **{nm: off})
            v = setup(place)
            ms = timeit(lambda: launch(plan, *v), reps=args.reps)
            diff = float((v[0] - want).abs().max())
            print(json.dumps({"rank": q, "buf": nm, "off": off, "bwd_ms": ms,
                              "max_abs_diff_vs_offset0": diff, "addr": addrs(*v)}), flush=True)
    # fresh plans (their internal buffers at new addresses), per-call buffers at offset 0
    keep = [plan]
    for i in range(args.plans):
        keep.append(mk.GraphPlan(pr, ix, vl, nloc, plan.num_edges, d, k, num_cols=ncol))
    malloc = os.environ.get("MAXK_PLAN_MALLOC", "default")
    for rnd in range(2):
        for i, p2 in enumerate(keep):
            ms = timeit(lambda: launch(p2, *ref), reps=args.reps)
            print(json.dumps({"rank": q, "plan": i, "round": rnd, "bwd_ms": ms, "malloc": malloc,
                              "plan_device_bytes": p2.device_bytes}), flush=True)


if __name__ == "__main__":
    main()
