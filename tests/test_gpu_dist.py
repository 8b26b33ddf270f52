"""GPU: the row-partitioned path of maxk_kernels.dist on one device.

* emulated W-rank partition: each rank's ShardedAggregation (a rectangular plan over the
  padded table of interleaved CBSR records) run on the GPU, the all-gather / reduce-scatter
  done with tensor ops; the union of the ranks' outputs must match the oracle on the whole
  graph; records gathered in place give bitwise the output of the contiguous tables;
* ShardedAggregation end to end over a real RCCL ("nccl") process group of world size 1.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

import maxk_kernels as mk
from maxk_kernels import graphs
from maxk_kernels.dist import RowPartition, ShardedAggregation
from oracle import oracle

pytestmark = pytest.mark.gpu


def _graph(n=6000, e=150_000, seed=41):
    p, i = graphs.synthetic_csr(n, e, seed=seed)
    return p, i, graphs.sage_mean_values(p)


def _fill_tables(part, sd, si, shard, gpu):
    """The all-gather emulated: every rank's rows and statistics pair in the shard's table."""
    world = part.world_size
    for r in range(world):
        ra, rb = part.rows(r)
        pos = part.table_positions(r, gpu)
        shard.table_data[pos] = sd[ra:rb]
        shard.table_index[pos] = si[ra:rb]
        sp = part.stats_position(r)
        mk.cbsr_stats(sd[ra:rb], si[ra:rb], out=shard.table_rec.view(torch.int32)[sp, :2])


@pytest.mark.parametrize("world,opts", [(2, None), (3, None), (8, None), (2, {"bwd_algo": 3}),
                                        (8, {"bwd_algo": 3}), (4, {"fwd_two_tables": 1}),
                                        (4, {"fwd_two_tables": 2}), (8, {"fwd_fixed": 2})])
@pytest.mark.parametrize("k", [8, 16, 32, 12])
def test_emulated_shards_match_oracle(gpu, world, opts, k):
    """ShardedAggregation as every rank builds it (one rectangular plan over the interleaved
    record table, a statistics pair in each rank's spare record), the all-gather emulated by
    filling each rank's table, the reduce-scatter by summing the ranks' partial gradients; the
    union of the ranks' outputs against the oracle on the whole graph. The forward gathers the
    records in place (no per-call pack) whatever table layout the plan would pick."""
    p, i, v = _graph()
    n, d = p.numel() - 1, 256
    od, oi = oracle.maxk(graphs.features(n, d, seed=15).numpy(), k)
    g = graphs.features(n, d, seed=16)
    ref_f, mag_f = oracle.spgemm_forward(p.numpy(), i.numpy(), v.numpy(), od, oi, d, with_mag=True)
    ref_b, mag_b = oracle.sspmm_backward(p.numpy(), i.numpy(), v.numpy(), g.numpy(), oi,
                                         with_mag=True)
    ptr, idx, val = p.to(gpu), i.to(gpu), v.to(gpu)
    sd, si, gg = torch.from_numpy(od).to(gpu), torch.from_numpy(oi).to(gpu), g.to(gpu)
    part = RowPartition(ptr, world)
    y = torch.empty((n, d), device=gpu)
    grad_sum = torch.zeros((part.padded_rows, k), device=gpu)
    for q in range(world):
        e0, e1 = part.edges(ptr, q)
        shard = ShardedAggregation(part, q, ptr, idx[e0:e1].clone(), val[e0:e1].clone(), d, k,
                                   plan_options=opts, local_edges=True)
        assert shard.stats
        a, b = part.rows(q)
        bd, bi = shard.local_buffers()
        h_q = graphs.features(n, d, seed=15)[a:b].contiguous().to(gpu)
        mk.maxk_forward(h_q, k, out=(bd, bi))               # top-k into the send records
        assert torch.equal(bd, sd[a:b]) and torch.equal(bi, si[a:b])
        shard._stage(bd, bi)
        pair = shard.send_rec[part.max_rows, :8].clone()    # cbsr_stats over the records
        bd2, bi2 = shard.local_topk(h_q)                    # statistics fused into the top-k
        assert torch.equal(bd2, sd[a:b]) and torch.equal(bi2, si[a:b])
        assert torch.equal(shard.send_rec[part.max_rows, :8], pair)
        shard._stage(bd2, bi2)                              # consumes the fused pair
        _fill_tables(part, sd, si, shard, gpu)
        # the rank's own statistics pair went out with its send records
        assert torch.equal(shard.send_rec[part.max_rows, :8],
                           shard.table_rec[part.stats_position(q), :8])
        y[a:b] = shard.compute_forward()
        grad_sum += shard.compute_backward(gg[a:b])
        del shard
    gs = torch.cat([grad_sum[part.table_positions(q, gpu)] for q in range(world)])
    ok, worst = oracle.close_enough(y.cpu().numpy(), ref_f, mag_f)
    assert ok, worst
    # per-rank partials summed in f32 (the reduce-scatter): the same bar
    ok, worst = oracle.close_enough(gs.cpu().numpy(), ref_b, mag_b)
    assert ok, worst


@pytest.mark.parametrize("k", [16, 32])
def test_records_in_place_equal_packed(gpu, k):
    """The forward over interleaved records (gathered in place) gives bitwise the output of the
    same plan over the two contiguous tables (packed per call or gathered as two tables), and
    the backward reading selectors at the record stride meets the oracle bar like the one
    reading sp_index (both backward algorithms)."""
    from maxk_kernels.dist import record_bytes, record_views
    p, i, v = _graph(n=5000, e=200_000, seed=44)
    n, d = p.numel() - 1, 256
    ptr, idx, val = p.to(gpu), i.to(gpu), v.to(gpu)
    x = graphs.features(n, d, seed=17).to(gpu)
    g = graphs.features(n, d, seed=18).to(gpu)
    sd, si = mk.maxk_forward(x, k, return_index=True)
    rec = torch.zeros((n, record_bytes(k)), dtype=torch.uint8, device=gpu)
    rd, ri = record_views(rec, k)
    mk.maxk_forward(x, k, out=(rd, ri))
    assert torch.equal(rd, sd) and torch.equal(ri, si)
    ref_b, mag_b = oracle.sspmm_backward(p.numpy(), i.numpy(), v.numpy(), g.cpu().numpy(),
                                         si.cpu().numpy(), with_mag=True)
    for opts in ({}, {"fwd_two_tables": 1}, {"fwd_two_tables": 2}, {"fwd_fixed": 2},
                 {"bwd_algo": 3}):
        plan = mk.GraphPlan(ptr, idx, val, n, i.numel(), d, k, options=opts)
        a = plan.forward(sd, si)
        b = plan.forward(rd, ri)
        torch.cuda.synchronize()
        assert torch.equal(a.view(torch.int32), b.view(torch.int32)), opts
        # (the column blocks' float CAS order varies from call to call: the oracle bar)
        for sel in (si, ri):
            ok, worst = oracle.close_enough(plan.backward(g, sel).cpu().numpy(), ref_b, mag_b)
            assert ok, (opts, worst)
    st = mk.cbsr_stats(rd, ri)
    assert torch.equal(st, mk.cbsr_stats(sd, si))


def test_forward_accumulate_vs_oracle(gpu):
    """maxk_spgemm_forward_acc: out += A densify(sp) on top of prior values."""
    p, i, v = _graph(n=3000, e=60_000, seed=43)
    n, d, k = p.numel() - 1, 256, 16
    x = graphs.features(n, d, seed=9)
    od, oi = oracle.maxk(x.numpy(), k)
    ref, mag = oracle.spgemm_forward(p.numpy(), i.numpy(), v.numpy(), od, oi, d, with_mag=True)
    prior = graphs.features(n, d, seed=10)
    ptr, idx, val = p.to(gpu), i.to(gpu), v.to(gpu)
    plan = mk.GraphPlan(ptr, idx, val, n, i.numel(), d, k)
    out = prior.clone().to(gpu)
    plan.forward(torch.from_numpy(od).to(gpu), torch.from_numpy(oi).to(gpu), out, accumulate=True)
    ok, worst = oracle.close_enough(out.cpu().numpy(), ref + prior.numpy(),
                                    mag + np.abs(prior.numpy()))
    assert ok, worst
    with pytest.raises(RuntimeError):
        plan.forward(torch.from_numpy(od).to(gpu), torch.from_numpy(oi).to(gpu), accumulate=True)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("opts", [None, {"bwd_algo": 3}])
def test_sharded_aggregation_rccl_world1(gpu, opts):
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=gpu)
    try:
        p, i, v = _graph(n=4000, e=90_000, seed=42)
        n, d, k = p.numel() - 1, 256, 16
        ptr, idx, val = p.to(gpu), i.to(gpu), v.to(gpu)
        x = graphs.features(n, d, seed=7).to(gpu)
        g = graphs.features(n, d, seed=8).to(gpu)
        sd, si = mk.maxk_forward(x, k, return_index=True)
        part = RowPartition(ptr, 1)
        shard = ShardedAggregation(part, 0, ptr, idx, val, d, k, plan_options=opts)
        y = shard.forward(sd, si)
        gs = shard.backward(g)
        od, oi = sd.cpu().numpy(), si.cpu().numpy()
        y_ref, y_mag = oracle.spgemm_forward(p.numpy(), i.numpy(), v.numpy(), od, oi, d,
                                             with_mag=True)
        g_ref, g_mag = oracle.sspmm_backward(p.numpy(), i.numpy(), v.numpy(), g.cpu().numpy(),
                                             oi, with_mag=True)
        torch.cuda.synchronize()
        ok, worst = oracle.close_enough(y.cpu().numpy(), y_ref, y_mag)
        assert ok, worst
        ok, worst = oracle.close_enough(gs.cpu().numpy(), g_ref, g_mag)
        assert ok, worst
        # top-k written straight into the send records (bench.py's N > 1 step): no copies
        sdb, sib = shard.local_buffers()
        r = mk.maxk_forward(x, k, return_index=True, out=(sdb, sib))
        assert r[0] is sdb and r[1] is sib
        assert torch.equal(sdb, sd) and torch.equal(sib, si)
        y2 = shard.forward(sdb, sib)
        torch.cuda.synchronize()
        ok, worst = oracle.close_enough(y2.cpu().numpy(), y_ref, y_mag)
        assert ok, worst
        with pytest.raises(RuntimeError):
            mk.maxk_forward(x, k, return_index=True, out=(sdb[:, :8], sib))
    finally:
        dist.destroy_process_group()
