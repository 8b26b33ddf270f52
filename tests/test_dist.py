"""CPU, world_size 2 (gloo): the row partition, the column remap into the padded
all-gather table and the two collectives of maxk_kernels.dist, with the oracle injected as
the per-rank compute (the GPU path runs the same class with the gfx950 kernels)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from maxk_kernels import graphs
from maxk_kernels.dist import RowPartition, ShardedAggregation


def test_partition_balances_nnz_and_remaps():
    ptr, idx = graphs.synthetic_csr(3000, 80_000, seed=7)
    for w in (1, 2, 3, 8):
        part = RowPartition(ptr, w)
        b = part.bounds
        assert int(b[0]) == 0 and int(b[-1]) == 3000 and bool((b[1:] >= b[:-1]).all())
        nnz = [int(ptr[part.rows(q)[1]] - ptr[part.rows(q)[0]]) for q in range(w)]
        assert sum(nnz) == 80_000
        assert max(nnz) - min(nnz) <= 2 * int((ptr[1:] - ptr[:-1]).max())
        for phases in (1, 2, 3):
            part = RowPartition(ptr, w, phases=phases)
            pos = part.remap_columns(torch.arange(3000, dtype=torch.int32))
            # the remap is injective into [0, padded_rows) and, per owner, order-preserving
            assert torch.unique(pos).numel() == 3000 and int(pos.max()) < part.padded_rows
            for q in range(w):
                a, b = part.rows(q)
                assert bool((pos[a + 1:b] > pos[a:b - 1]).all())
                assert torch.equal(part.table_positions(q), pos[a:b].long())
            if phases == 1:
                assert bool((pos[1:] > pos[:-1]).all())
                # each rank's block ends in a spare (statistics) row no node maps to
                spare = torch.tensor([part.stats_position(q) for q in range(w)])
                assert not bool(torch.isin(spare, pos.long()).any())
                assert part.padded_rows == w * (part.max_rows + 1)
            # a phase's CSR keeps exactly the edges whose column lies in that phase
            lp, li, lv = part.local_csr(ptr, idx, graphs.sage_mean_values(ptr), 0)
            tot = 0
            for ph in range(phases):
                pp, pi, pv = part.phase_csr(lp, li, lv, ph)
                assert int(pp[-1]) == pi.numel() == pv.numel()
                assert pi.numel() == 0 or (int(pi.min()) >= 0 and int(pi.max()) < part.phase_cols)
                tot += pi.numel()
            assert tot == li.numel()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, ret, phases=1, size=(700, 15_000), split=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle
        (n, e), d, k = size, 32, 8
        ptr, idx = graphs.synthetic_csr(n, e, seed=3)
        val = graphs.sage_mean_values(ptr)
        x = graphs.features(n, d, seed=1)
        g = graphs.features(n, d, seed=2)
        part = RowPartition(ptr, world, phases=phases)
        r0, r1 = part.rows(rank)
        sd, si = oracle.maxk(x[r0:r1].numpy(), k)

        def part_graph(i):
            # part i's CSR (a column phase, or the own / remote columns of the split); the
            # oracle indexes CBSR rows by column id: pad the local rows to the table size
            lptr, lidx, lval, nc = shard.parts[i]
            nr = max(nc, r1 - r0)
            full_ptr = np.full(nr + 1, lptr[-1].item(), np.int32)
            full_ptr[: lptr.numel()] = lptr.numpy()
            return full_ptr, lidx.numpy(), lval.numpy(), nr, nc

        def fwd(i, td, ti, out):
            fp, li, lv, nr, nc = part_graph(i)
            assert td.shape[0] == nc
            tdp = np.zeros((nr, k), np.float32)
            tip = np.zeros((nr, k), np.uint8)
            tdp[:nc], tip[:nc] = td.numpy(), ti.numpy()
            y = torch.from_numpy(oracle.spgemm_forward(fp, li, lv, tdp, tip, d)[: r1 - r0].copy())
            return y if out is None else out + y

        def bwd(i, gl, ti):
            fp, li, lv, nr, nc = part_graph(i)
            gfull = np.zeros((nr, d), np.float32)
            gfull[: r1 - r0] = gl.numpy()
            tip = np.zeros((nr, k), np.uint8)
            tip[:nc] = ti.numpy()
            return torch.from_numpy(oracle.sspmm_backward(fp, li, lv, gfull, tip)[:nc].copy())

        shard = ShardedAggregation(part, rank, ptr, idx, val, d, k, fwd=fwd, bwd=bwd,
                                   split=split)
        if split:   # the own-column part holds exactly the edges into this rank's rows
            own = ((idx[int(ptr[r0]):int(ptr[r1])] >= r0) & (idx[int(ptr[r0]):int(ptr[r1])] < r1))
            assert shard.parts[0][1].numel() == int(own.sum())
            assert shard.parts[0][1].numel() + shard.parts[1][1].numel() == int(ptr[r1] - ptr[r0])
        y = shard.forward(torch.from_numpy(sd), torch.from_numpy(si))
        gs = shard.backward(g[r0:r1])
        ret[rank] = (r0, r1, y.numpy().copy(), gs.numpy().copy(),
                     shard.unpad_table(shard.table_index).numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,phases,size,split", [
    (2, 1, (700, 15_000), False), (2, 2, (700, 15_000), False), (3, 2, (700, 15_000), False),
    (4, 1, (20_000, 600_000), False),
    # local-columns-first split: own-column edges from the send buffers (overlapping the
    # all-gather), remote edges accumulated on the table; the backward over all edges
    (2, 1, (700, 15_000), True), (3, 1, (700, 15_000), True), (4, 1, (20_000, 600_000), True)])
def test_sharded_aggregation_matches_single(world, phases, size, split):
    from oracle import oracle
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), ret, phases, size, split), nprocs=world,
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
        r0, r1, y, gs, table_index = ret[rank]
        assert np.array_equal(table_index, si)            # the all-gather reassembles CBSR
        ok, worst = oracle.close_enough(y, y_ref[r0:r1], y_mag[r0:r1])
        assert ok, worst
        ok, worst = oracle.close_enough(gs, g_ref[r0:r1], g_mag[r0:r1])
        assert ok, worst
