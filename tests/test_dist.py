"""CPU, world sizes 2-4 (gloo): the row partition, the column remap into the padded
all-gather table of interleaved CBSR records and the two collectives of maxk_kernels.dist (one
all-gather, one reduce-scatter), with the oracle injected as the per-rank compute (the GPU path
runs the same class with the gfx950 kernels); and the per-rank graph generation bench.py uses."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from maxk_kernels import graphs
from maxk_kernels.dist import RowPartition, ShardedAggregation, record_bytes, record_views


def test_partition_balances_nnz_and_remaps():
    ptr, idx = graphs.synthetic_csr(3000, 80_000, seed=7)
    for w in (1, 2, 3, 8):
        part = RowPartition(ptr, w)
        b = part.bounds
        assert int(b[0]) == 0 and int(b[-1]) == 3000 and bool((b[1:] >= b[:-1]).all())
        nnz = [int(ptr[part.rows(q)[1]] - ptr[part.rows(q)[0]]) for q in range(w)]
        assert sum(nnz) == 80_000
        assert max(nnz) - min(nnz) <= 2 * int((ptr[1:] - ptr[:-1]).max())
        pos = part.remap_columns(torch.arange(3000, dtype=torch.int32))
        # the remap is injective into [0, padded_rows), order-preserving
        assert torch.unique(pos).numel() == 3000 and int(pos.max()) < part.padded_rows
        assert bool((pos[1:] > pos[:-1]).all())
        for q in range(w):
            a, b2 = part.rows(q)
            assert torch.equal(part.table_positions(q), pos[a:b2].long())
        # each rank's block ends in a spare (statistics) row no node maps to
        spare = torch.tensor([part.stats_position(q) for q in range(w)])
        assert not bool(torch.isin(spare, pos.long()).any())
        assert part.padded_rows == w * (part.max_rows + 1)
        # a rank's own edges, sliced or given as they are, give the same local CSR
        val = graphs.sage_mean_values(ptr)
        for q in range(w):
            e0, e1 = part.edges(ptr, q)
            full = part.local_csr(ptr, idx, val, q)
            own = part.local_csr(ptr, idx[e0:e1], val[e0:e1], q, local_edges=True)
            assert all(torch.equal(x, y) for x, y in zip(full, own))


def test_record_layout_views():
    """Interleaved CBSR records {k f32 values, k u8 selectors (padded to whole words)}: the
    strided views read and write exactly the record bytes."""
    for k in (8, 16, 32, 5, 6):
        rb = record_bytes(k)
        assert rb % 4 == 0 and rb >= 5 * k and (k % 4 != 0 or rb == 5 * k)
        buf = torch.zeros((7, rb), dtype=torch.uint8)
        d, i = record_views(buf, k)
        assert d.shape == (7, k) and i.shape == (7, k) and d.stride(1) == 1 and i.stride(1) == 1
        d[3] = torch.arange(k, dtype=torch.float32) + 1.5
        i[3] = torch.arange(k, dtype=torch.uint8) * 3
        row = buf[3]
        assert torch.equal(row[:4 * k].view(torch.float32), torch.arange(k, dtype=torch.float32) + 1.5)
        assert torch.equal(row[4 * k:5 * k], torch.arange(k, dtype=torch.uint8) * 3)
        assert not buf[2].any() and not buf[4].any()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, ret, size=(700, 15_000), local_edges=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle
        (n, e), d, k = size, 32, 8
        ptr, idx = graphs.synthetic_csr(n, e, seed=3)
        val = graphs.sage_mean_values(ptr)
        x = graphs.features(n, d, seed=1)
        g = graphs.features(n, d, seed=2)
        part = RowPartition(ptr, world)
        r0, r1 = part.rows(rank)
        sd, si = oracle.maxk(x[r0:r1].numpy(), k)
        nc = part.padded_rows
        nr = max(nc, r1 - r0)

        def full_ptr():
            # the oracle indexes CBSR rows by column id: pad the local rows to the table size
            lptr = shard.ptr
            fp = np.full(nr + 1, lptr[-1].item(), np.int32)
            fp[: lptr.numel()] = lptr.numpy()
            return fp

        def fwd(td, ti, out=None):
            assert td.shape[0] == nc and td.stride(0) == record_bytes(k) // 4   # records
            tdp = np.zeros((nr, k), np.float32)
            tip = np.zeros((nr, k), np.uint8)
            tdp[:nc], tip[:nc] = td.numpy(), ti.numpy()
            return torch.from_numpy(oracle.spgemm_forward(full_ptr(), shard.idx.numpy(),
                                                          shard.val.numpy(), tdp, tip,
                                                          d)[: r1 - r0].copy())

        def bwd(gl, ti):
            gfull = np.zeros((nr, d), np.float32)
            gfull[: r1 - r0] = gl.numpy()
            tip = np.zeros((nr, k), np.uint8)
            tip[:nc] = ti.numpy()
            return torch.from_numpy(oracle.sspmm_backward(full_ptr(), shard.idx.numpy(),
                                                          shard.val.numpy(), gfull, tip)[:nc].copy())

        if local_edges:   # the rank holds only its own rows' edges (bench.py's N > 1 setup)
            e0, e1 = part.edges(ptr, rank)
            shard = ShardedAggregation(part, rank, ptr, idx[e0:e1].clone(), val[e0:e1].clone(),
                                       d, k, fwd=fwd, bwd=bwd, local_edges=True)
        else:
            shard = ShardedAggregation(part, rank, ptr, idx, val, d, k, fwd=fwd, bwd=bwd)
        # the top-k straight into the send records, as bench.py writes it
        bd, bi = shard.local_buffers()
        bd.copy_(torch.from_numpy(sd))
        bi.copy_(torch.from_numpy(si))
        y = shard.forward(bd, bi)
        gs = shard.backward(g[r0:r1])
        ret[rank] = (r0, r1, y.numpy().copy(), gs.numpy().copy(),
                     shard.unpad_table(shard.table_index).numpy().copy(),
                     shard.unpad_table(shard.table_data).numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,size,local_edges", [
    (2, (700, 15_000), False), (3, (700, 15_000), False), (2, (700, 15_000), True),
    (4, (20_000, 600_000), False), (4, (20_000, 600_000), True)])
def test_sharded_aggregation_matches_single(world, size, local_edges):
    from oracle import oracle
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), ret, size, local_edges), nprocs=world,
             join=True)
    (n, e), d, k = size, 32, 8
    ptr, idx = graphs.synthetic_csr(n, e, seed=3)
    val = graphs.sage_mean_values(ptr)
    x = graphs.features(n, d, seed=1).numpy()
    g = graphs.features(n, d, seed=2).numpy()
    sd, si = oracle.maxk(x, k)
    y_ref, y_mag = oracle.spgemm_forward(ptr.numpy(), idx.numpy(), val.numpy(), sd, si, d,
                                         with_mag=True)
    g_ref, g_mag = oracle.sspmm_backward(ptr.numpy(), idx.numpy(), val.numpy(), g, si,
                                         with_mag=True)
    for rank in range(world):
        r0, r1, y, gs, table_index, table_data = ret[rank]
        assert np.array_equal(table_index, si)            # the all-gather reassembles CBSR
        assert np.array_equal(table_data, sd)
        ok, worst = oracle.close_enough(y, y_ref[r0:r1], y_mag[r0:r1])
        assert ok, worst
        ok, worst = oracle.close_enough(gs, g_ref[r0:r1], g_mag[r0:r1])
        assert ok, worst


def test_rank_rows_generate_the_same_graph():
    """bench.py's graph: each rank generates only its rows (counter-based draws) and gets
    exactly those rows of the whole graph, for every world size."""
    ptr = graphs.synthetic_ptr(6000, 300_000, seed=97)
    full = graphs.synthetic_rows(ptr, 97)
    assert full.numel() == int(ptr[-1]) == 300_000
    p = ptr.long()
    d = p[1:] - p[:-1]
    rows = torch.repeat_interleave(torch.arange(6000), d)
    # sorted, distinct columns per row, each row with its self-loop
    key = rows * 6000 + full.long()
    assert bool((key[1:] > key[:-1]).all())
    assert int((full.long() == rows).sum()) == 6000
    for w in (2, 3, 8):
        part = RowPartition(ptr, w)
        got = torch.cat([graphs.synthetic_rows(ptr, 97, part.rows(q)) for q in range(w)])
        assert torch.equal(got, full)
