"""GPU: the row-partitioned path of maxk_kernels.dist on one device.

* emulated W-rank partition: each rank's rectangular plan (columns remapped into the padded
  all-gather table) run on the GPU, the all-gather / reduce-scatter done with tensor ops;
  the union of the ranks' outputs must match the oracle on the whole graph;
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


@pytest.mark.parametrize("world,phases,opts", [(2, 1, None), (3, 1, None), (8, 1, None),
                                               (2, 2, None), (8, 2, None), (3, 3, None),
                                               (2, 1, {"bwd_algo": 3}), (8, 2, {"bwd_algo": 3})])
@pytest.mark.parametrize("k", [16, 32])
def test_emulated_partition_matches_oracle(gpu, world, phases, opts, k):
    """Every rank's per-phase rectangular plans (columns remapped into the phase-major
    padded table) on one GPU; the all-gather / reduce-scatter done with tensor ops; also
    with the two-pass backward forced on every shard."""
    p, i, v = _graph()
    n, d = p.numel() - 1, 256
    x = graphs.features(n, d, seed=5)
    g = graphs.features(n, d, seed=6)
    od, oi = oracle.maxk(x.numpy(), k)
    ref_f, mag_f = oracle.spgemm_forward(p.numpy(), i.numpy(), v.numpy(), od, oi, d, with_mag=True)
    ref_b, mag_b = oracle.sspmm_backward(p.numpy(), i.numpy(), v.numpy(), g.numpy(), oi,
                                         with_mag=True)
    ptr, idx, val = p.to(gpu), i.to(gpu), v.to(gpu)
    part = RowPartition(ptr, world, phases=phases)
    # the padded all-gather table every rank would hold
    table_d = torch.zeros((part.padded_rows, k), device=gpu)
    table_i = torch.zeros((part.padded_rows, k), dtype=torch.uint8, device=gpu)
    for q in range(world):
        a, b = part.rows(q)
        pos = part.table_positions(q, gpu)
        table_d[pos] = torch.from_numpy(od[a:b]).to(gpu)
        table_i[pos] = torch.from_numpy(oi[a:b]).to(gpu)
    y = torch.empty((n, d), device=gpu)
    grad_table = torch.zeros((part.padded_rows, k), device=gpu)
    nc = part.phase_cols
    for q in range(world):
        a, b = part.rows(q)
        lp, li, lv = part.local_csr(ptr, idx, val, q)
        out = torch.empty((b - a, d), device=gpu)
        for ph in range(phases):
            pp, pi, pv = part.phase_csr(lp, li, lv, ph)
            plan = mk.GraphPlan(pp, pi, pv, b - a, pi.numel(), d, k, num_cols=nc, options=opts)
            if opts and pi.numel() > 0:
                assert plan.info()["bwd_algo"] == 3
            plan.forward(table_d[ph * nc:(ph + 1) * nc], table_i[ph * nc:(ph + 1) * nc], out,
                         accumulate=ph > 0)
            grad_table[ph * nc:(ph + 1) * nc] += plan.backward(                # reduce-scatter
                g[a:b].contiguous().to(gpu), table_i[ph * nc:(ph + 1) * nc])
        y[a:b] = out
    gs = torch.cat([grad_table[part.table_positions(q, gpu)] for q in range(world)])
    ok, worst = oracle.close_enough(y.cpu().numpy(), ref_f, mag_f)
    assert ok, worst
    # per-rank partials summed in f32 (the reduce-scatter): the same bar
    ok, worst = oracle.close_enough(gs.cpu().numpy(), ref_b, mag_b)
    assert ok, worst


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("split", [False, True])
@pytest.mark.parametrize("k", [16, 32])
def test_emulated_shards_stats_and_split(gpu, world, split, k):
    """ShardedAggregation as every rank builds it (statistics row in each rank's block; the
    local-columns-first split), the all-gather emulated by filling each rank's table and
    statistics rows, the reduce-scatter by summing the ranks' partial gradients."""
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
        shard = ShardedAggregation(part, q, ptr, idx, val, d, k, split=split)
        assert shard.stats and len(shard.plans) == (3 if split else 1)
        a, b = part.rows(q)
        shard._stage(sd[a:b], si[a:b])
        for r in range(world):
            ra, rb = part.rows(r)
            pos = part.table_positions(r, gpu)
            shard.table_data[pos] = sd[ra:rb]
            shard.table_index[pos] = si[ra:rb]
            sp = part.stats_position(r)
            shard.table_data[sp] = 0.0
            shard.table_index[sp] = 0
            mk.cbsr_stats(sd[ra:rb], si[ra:rb], out=shard.stats_words(shard.table_index, sp))
        # the rank's own statistics row went out with its send buffer; its values stay zero
        assert torch.equal(shard.send_index[part.rows_per_phase],
                           shard.table_index[part.stats_position(q)])
        assert not shard.send_data[part.rows_per_phase].any()
        y[a:b] = shard.compute_forward()
        gl = gg[a:b].contiguous()
        grad_sum += shard._bwd(2 if split else 0, gl, shard.table_index)
        del shard
    gs = torch.cat([grad_sum[part.table_positions(q, gpu)] for q in range(world)])
    ok, worst = oracle.close_enough(y.cpu().numpy(), ref_f, mag_f)
    assert ok, worst
    ok, worst = oracle.close_enough(gs.cpu().numpy(), ref_b, mag_b)
    assert ok, worst


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


@pytest.mark.parametrize("phases,opts,split", [(1, None, False), (2, None, False),
                                               (1, {"bwd_algo": 3}, False), (1, None, True)])
def test_sharded_aggregation_rccl_world1(gpu, phases, opts, split):
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
        part = RowPartition(ptr, 1, phases=phases)
        shard = ShardedAggregation(part, 0, ptr, idx, val, d, k, plan_options=opts, split=split)
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
        # top-k written straight into the send buffers (bench.py's N > 1 step): no copies
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
