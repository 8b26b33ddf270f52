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
        pos = part.remap_columns(torch.arange(3000, dtype=torch.int32))
        # the remap is injective into [0, padded_rows) and order-preserving per owner
        assert torch.unique(pos).numel() == 3000 and int(pos.max()) < part.padded_rows
        assert bool((pos[1:] > pos[:-1]).all())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, ret):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle
        n, d, k = 700, 32, 8
        ptr, idx = graphs.synthetic_csr(n, 15_000, seed=3)
        val = graphs.sage_mean_values(ptr)
        x = graphs.features(n, d, seed=1)
        g = graphs.features(n, d, seed=2)
        part = RowPartition(ptr, world)
        r0, r1 = part.rows(rank)
        sd, si = oracle.maxk(x[r0:r1].numpy(), k)

        def fwd(td, ti):
            lptr, lidx, lval = shard.ptr, shard.idx, shard.val
            # oracle reads CBSR rows by column id; pad local rows to padded_rows
            full_ptr = np.full(part.padded_rows + 1, lptr[-1].item(), np.int32)
            full_ptr[: lptr.numel()] = lptr.numpy()
            y = oracle.spgemm_forward(full_ptr, lidx.numpy(), lval.numpy(), td.numpy(),
                                      ti.numpy(), d)
            return torch.from_numpy(y[: r1 - r0].copy())

        def bwd(gl, ti):
            lptr, lidx, lval = shard.ptr, shard.idx, shard.val
            full_ptr = np.full(part.padded_rows + 1, lptr[-1].item(), np.int32)
            full_ptr[: lptr.numel()] = lptr.numpy()
            gfull = np.zeros((part.padded_rows, d), np.float32)
            gfull[: r1 - r0] = gl.numpy()
            return torch.from_numpy(oracle.sspmm_backward(full_ptr, lidx.numpy(), lval.numpy(),
                                                          gfull, ti.numpy()))

        shard = ShardedAggregation(part, rank, ptr, idx, val, d, k, fwd=fwd, bwd=bwd)
        y = shard.forward(torch.from_numpy(sd), torch.from_numpy(si))
        gs = shard.backward(g[r0:r1])
        ret[rank] = (r0, r1, y.numpy().copy(), gs.numpy().copy(),
                     shard.unpad_table(shard.table_index).numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_aggregation_matches_single(world):
    from oracle import oracle
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), ret), nprocs=world, join=True)
    n, d, k = 700, 32, 8
    ptr, idx = graphs.synthetic_csr(n, 15_000, seed=3)
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
