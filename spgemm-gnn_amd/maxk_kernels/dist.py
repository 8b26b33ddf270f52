"""Row-partitioned MaxK aggregation over several GPUs of one node (one process per GPU).

The reference is single-GPU (no NCCL / torch.distributed anywhere; multi-GPU is future
work in README_INTEGRATED.md:382). The path shards by destination rows with one real
exchange per direction:

* partition: contiguous row ranges balanced by nnz; rank q owns rows [start_q, end_q),
  their CSR slice (columns keep pointing at any node) and computes the top-k of its own
  rows (weights are replicated);
* forward : RCCL all-gathers of the k-sparse CBSR block (sp_data f32 and sp_index u8,
  coalesced into one group call) straight into the tables the kernels read, padded to
  W x max_rows rows; the rank's top-k can be written directly into its send buffers
  (``local_buffers``), so the exchange moves no extra copies. Then the local SpGEMM over
  the rank's rows with a rectangular plan whose column ids are remapped into that padded
  table (remapping is done once, at partition time);
* backward: the local SSpMM produces a partial grad_sp for every (padded) column; an
  RCCL reduce-scatter (sum) returns each rank its own rows' gradient.

Bytes exchanged per step are 5kN (all-gathers) + 4kN (reduce-scatter), i.e. 18.6 MB +
14.9 MB for Reddit at k=16, against 238 MB for all-gathering dense features.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist


class RowPartition:
    """Contiguous destination-row ranges with ~equal nnz per rank."""

    def __init__(self, ptr: torch.Tensor, world_size: int):
        p = ptr.detach().to("cpu", torch.int64)
        n = p.numel() - 1
        e = int(p[-1])
        w = int(world_size)
        targets = torch.tensor([(e * q) // w for q in range(w + 1)], dtype=torch.int64)
        b = torch.searchsorted(p, targets, right=False).clamp_(max=n)
        b[0], b[-1] = 0, n
        b = torch.cummax(b, 0).values
        self.world_size = w
        self.num_nodes = n
        self.num_edges = e
        self.bounds = b                      # [W+1] row boundaries
        counts = b[1:] - b[:-1]
        self.max_rows = max(1, int(counts.max()))
        self.padded_rows = w * self.max_rows

    def rows(self, rank: int):
        return int(self.bounds[rank]), int(self.bounds[rank + 1])

    def remap_columns(self, idx: torch.Tensor) -> torch.Tensor:
        """Global column id -> position in the padded all-gather table."""
        b = self.bounds.to(idx.device)
        c = idx.to(torch.int64)
        q = torch.searchsorted(b, c, right=True) - 1
        return (q * self.max_rows + (c - b[q])).to(torch.int32)

    def local_csr(self, ptr: torch.Tensor, idx: torch.Tensor, val: torch.Tensor, rank: int):
        """(ptr, remapped idx, val) of rank's rows; ptr rebased to 0."""
        r0, r1 = self.rows(rank)
        e0, e1 = int(ptr[r0]), int(ptr[r1])
        lptr = (ptr[r0:r1 + 1].to(torch.int64) - e0).to(torch.int32).contiguous()
        lidx = self.remap_columns(idx[e0:e1]).contiguous()
        lval = val[e0:e1].contiguous()
        return lptr, lidx, lval


FwdFn = Callable[[torch.Tensor, torch.Tensor], torch.Tensor]
BwdFn = Callable[[torch.Tensor, torch.Tensor], torch.Tensor]


class ShardedAggregation:
    """One rank's share of Y = A densify(sp) and of its SSpMM backward.

    ``fwd(table_data, table_index) -> out_local`` and ``bwd(grad_out_local, table_index)
    -> grad_table`` default to the gfx950 kernels through a rectangular GraphPlan; tests
    on CPU (gloo) inject checker callables to exercise the partition and the collectives.
    """

    def __init__(self, part: RowPartition, rank: int, ptr: torch.Tensor, idx: torch.Tensor,
                 val: torch.Tensor, dim_origin: int, dim_k: int,
                 group: Optional[dist.ProcessGroup] = None, fwd: Optional[FwdFn] = None,
                 bwd: Optional[BwdFn] = None):
        self.part, self.rank, self.group = part, rank, group
        self.dim_origin, self.dim_k = int(dim_origin), int(dim_k)
        self.r0, self.r1 = part.rows(rank)
        self.n_local = self.r1 - self.r0
        self.ptr, self.idx, self.val = part.local_csr(ptr, idx, val, rank)
        dev = self.ptr.device
        m, k = part.max_rows, self.dim_k
        # padded send buffers (rows >= n_local stay zero) and the all-gathered tables
        self.send_data = torch.zeros((m, k), dtype=torch.float32, device=dev)
        self.send_index = torch.zeros((m, k), dtype=torch.uint8, device=dev)
        self.table_data = torch.empty((part.padded_rows, k), dtype=torch.float32, device=dev)
        self.table_index = torch.empty((part.padded_rows, k), dtype=torch.uint8, device=dev)
        self.grad_local = torch.empty((m, k), dtype=torch.float32, device=dev)
        self.plan = None
        if fwd is None or bwd is None:
            from .ops import GraphPlan
            self.plan = GraphPlan(self.ptr, self.idx, self.val, self.n_local, self.idx.numel(),
                                  self.dim_origin, self.dim_k, num_cols=part.padded_rows)
        self._fwd = fwd or (lambda d, i: self.plan.forward(d, i))
        self._bwd = bwd or (lambda g, i: self.plan.backward(g, i))

    def local_buffers(self):
        """(sp_data, sp_index) views [n_local, k] of the send buffers: write this rank's
        top-k here (``maxk_forward(h, k, out=...)``) and ``gather`` sends them as they are."""
        return self.send_data[: self.n_local], self.send_index[: self.n_local]

    def gather(self, sp_data_local: torch.Tensor, sp_index_local: torch.Tensor) -> None:
        """All-gather this rank's CBSR rows into the padded tables (RCCL over xGMI)."""
        n = self.n_local
        if sp_data_local.data_ptr() != self.send_data.data_ptr():
            self.send_data[:n].copy_(sp_data_local)
        if sp_index_local.data_ptr() != self.send_index.data_ptr():
            self.send_index[:n].copy_(sp_index_local)
        cm = getattr(dist, "_coalescing_manager", None)
        if cm is not None and self.table_data.is_cuda:
            with cm(group=self.group, device=self.table_data.device):
                dist.all_gather_into_tensor(self.table_data, self.send_data, group=self.group)
                dist.all_gather_into_tensor(self.table_index, self.send_index, group=self.group)
        else:
            dist.all_gather_into_tensor(self.table_data, self.send_data, group=self.group)
            dist.all_gather_into_tensor(self.table_index, self.send_index, group=self.group)

    def forward(self, sp_data_local: torch.Tensor, sp_index_local: torch.Tensor) -> torch.Tensor:
        self.gather(sp_data_local, sp_index_local)
        return self._fwd(self.table_data, self.table_index)

    def backward(self, grad_out_local: torch.Tensor) -> torch.Tensor:
        grad_table = self._bwd(grad_out_local.contiguous(), self.table_index)
        dist.reduce_scatter_tensor(self.grad_local, grad_table, op=dist.ReduceOp.SUM,
                                   group=self.group)
        return self.grad_local[: self.n_local]

    def unpad_table(self, table: torch.Tensor) -> torch.Tensor:
        """Padded [W*max_rows, ...] table -> natural node order [N, ...] (tests/inspection)."""
        parts = []
        for q in range(self.part.world_size):
            a, b = self.part.rows(q)
            parts.append(table[q * self.part.max_rows: q * self.part.max_rows + (b - a)])
        return torch.cat(parts)
