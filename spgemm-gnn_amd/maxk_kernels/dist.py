"""Row-partitioned MaxK aggregation over several GPUs of one node (one process per GPU).

The reference is single-GPU (no NCCL / torch.distributed anywhere; multi-GPU is future
work in README_INTEGRATED.md:382). The path shards by destination rows with one real
exchange per direction:

* partition: contiguous row ranges balanced by nnz; rank q owns rows [start_q, end_q),
  their CSR slice (columns keep pointing at any node) and computes the top-k of its own
  rows (weights are replicated);
* forward : ONE RCCL all-gather of the k-sparse CBSR block as interleaved records
  {k f32 values, k u8 selectors} per row (5k bytes at k % 4 == 0), straight into the table
  the kernels read: the forward gathers these records in place (no per-call record pack over
  the N columns; maxk_spgemm_forward_tables), except at k = 16, where the plan's pair-chunk
  layout repacks them in one pass without statistics (W = 8 shard 0.356 against
  0.358 ms in place), and the backward reads the selectors at the record stride. The rank's top-k is written straight into its send records
  (``local_buffers`` + maxk_topk_cbsr_tables), so the exchange moves no extra copies. Then
  the local SpGEMM over the rank's rows with a rectangular plan whose column ids are
  remapped into the gathered table (once, at partition time);
* backward: the local SSpMM produces a partial grad_sp for every (padded) column; an RCCL
  reduce-scatter (sum) returns each rank its own rows' gradient.

Fixed-point statistics: every rank's block of the table ends in a spare row no edge points
at. Before the all-gather the rank writes the fixed-point statistics of its own rows into the
first 8 bytes of that record (``maxk_cbsr_stats``: two words), the gathered table carries one
pair per rank and the forward reads those W pairs (``maxk_spgemm_forward_ex``) instead of
scanning the whole table.

The spare rows (``RowPartition.stats_position``) are therefore NOT CBSR data: their first two
"values" are statistics words. No edge reads them, so the shard's own forward and backward are
unaffected, but a pass over the whole gathered table would take those bit patterns for values:
``cbsr_stats(shard.table_data, ...)`` or a ``GraphPlan.forward`` on the shard's tables without
``stats=`` (its own statistics pass would count the spare rows, coarsening the fixed-point
scale or falling back to f64). Use ``ShardedAggregation.forward`` / ``compute_forward`` (they
pass the per-rank pairs) and ``unpad_table`` (node rows only) for such passes.

Bytes exchanged per step are 5kN (all-gather) + 4kN (reduce-scatter), i.e. 18.6 MB + 14.9 MB
for Reddit at k=16, against 238 MB for all-gathering dense features. Round 3's two
all-gathers (values, selectors), column phases and local-columns-first split are gone: the
phases and the split cost more compute than the exchange they could hide.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist


def record_bytes(k: int) -> int:
    """Bytes of one interleaved CBSR record: k f32 values, then the k selector bytes padded to
    whole words (5k at k % 4 == 0)."""
    return 4 * k + 4 * (-(-k // 4))


def record_views(buf: torch.Tensor, k: int):
    """(values f32 [rows, k], selectors u8 [rows, k]) strided views of a uint8 record buffer
    [rows, record_bytes(k)]."""
    rb = record_bytes(k)
    assert buf.dtype == torch.uint8 and buf.dim() == 2 and buf.shape[1] == rb
    return buf[:, :4 * k].view(torch.float32), buf[:, 4 * k:4 * k + k]


class RowPartition:
    """Contiguous destination-row ranges with ~equal nnz per rank, and the layout of the
    all-gathered record table: rank q's block holds its rows at [q * block_rows, ...) and
    ends in a spare row carrying its fixed-point statistics."""

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
        self.block_rows = self.max_rows + 1  # + the statistics row
        self.padded_rows = w * self.block_rows

    def rows(self, rank: int):
        return int(self.bounds[rank]), int(self.bounds[rank + 1])

    def edges(self, ptr: torch.Tensor, rank: int):
        """CSR edge range [e0, e1) of rank's rows."""
        r0, r1 = self.rows(rank)
        return int(ptr[r0]), int(ptr[r1])

    def remap_columns(self, idx: torch.Tensor) -> torch.Tensor:
        """Global column id -> position in the padded all-gather table."""
        b = self.bounds.to(idx.device)
        c = idx.to(torch.int64)
        q = torch.searchsorted(b, c, right=True) - 1
        return (q * self.block_rows + (c - b[q])).to(torch.int32)

    def table_positions(self, rank: int, device=None) -> torch.Tensor:
        """Table rows holding rank's nodes, in node order (int64 [n_rank])."""
        a, b = self.rows(rank)
        return rank * self.block_rows + torch.arange(b - a, dtype=torch.int64, device=device)

    def stats_position(self, rank: int) -> int:
        """Table row of rank's statistics pair."""
        return rank * self.block_rows + self.max_rows

    def local_csr(self, ptr: torch.Tensor, idx: torch.Tensor, val: torch.Tensor, rank: int,
                  local_edges: bool = False):
        """(ptr rebased to 0, remapped idx, val) of rank's rows. ``local_edges``: idx / val
        already hold only those rows' edges (a rank that generated or loaded its own rows)."""
        r0, r1 = self.rows(rank)
        e0, e1 = int(ptr[r0]), int(ptr[r1])
        lptr = (ptr[r0:r1 + 1].to(torch.int64) - e0).to(torch.int32).contiguous()
        if not local_edges:
            idx, val = idx[e0:e1], val[e0:e1]
        assert idx.numel() == e1 - e0 and val.numel() == e1 - e0, "edges of the wrong rows"
        return lptr, self.remap_columns(idx).contiguous(), val.contiguous()


# injected per-rank compute (CPU tests): fwd(table_data, table_index, out=None) -> out [n_local,
# D]; bwd(grad_out [n_local, D], table_index) -> grad for every table row [padded_rows, k].
FwdFn = Callable[[torch.Tensor, torch.Tensor], torch.Tensor]
BwdFn = Callable[[torch.Tensor, torch.Tensor], torch.Tensor]


class ShardedAggregation:
    """One rank's share of Y = A densify(sp) and of its SSpMM backward.

    ``fwd``/``bwd`` default to the gfx950 kernels through one rectangular GraphPlan
    (``plan_options``: the same knobs as ``GraphPlan(options=...)``, e.g.
    ``{"bwd_algo": 3}``); tests on CPU (gloo) inject checker callables to exercise the
    partition, the record layout and the collectives.
    """

    def __init__(self, part: RowPartition, rank: int, ptr: torch.Tensor, idx: torch.Tensor,
                 val: torch.Tensor, dim_origin: int, dim_k: int,
                 group: Optional[dist.ProcessGroup] = None, fwd: Optional[FwdFn] = None,
                 bwd: Optional[BwdFn] = None, plan_options: Optional[dict] = None,
                 local_edges: bool = False):
        self.part, self.rank, self.group = part, rank, group
        self.dim_origin, self.dim_k = int(dim_origin), int(dim_k)
        self.r0, self.r1 = part.rows(rank)
        self.n_local = self.r1 - self.r0
        self.ptr, self.idx, self.val = part.local_csr(ptr, idx, val, rank, local_edges)
        dev = self.ptr.device
        k = self.dim_k
        rb = record_bytes(k)
        # send block (rows >= n_local stay zero; the last row carries the statistics) and the
        # all-gathered table, both interleaved records
        self.send_rec = torch.zeros((part.block_rows, rb), dtype=torch.uint8, device=dev)
        self.table_rec = torch.zeros((part.padded_rows, rb), dtype=torch.uint8, device=dev)
        self.send_data, self.send_index = record_views(self.send_rec, k)
        # rows stats_position(q) of these views are the spare statistics records, not CBSR data
        self.table_data, self.table_index = record_views(self.table_rec, k)
        self.grad_table = torch.empty((part.padded_rows, k), dtype=torch.float32, device=dev)
        self.grad_local = torch.empty((part.block_rows, k), dtype=torch.float32, device=dev)
        self.plan = None
        native = fwd is None or bwd is None
        if native:
            from .ops import GraphPlan
            self.plan = GraphPlan(self.ptr, self.idx, self.val, self.n_local, self.idx.numel(),
                                  self.dim_origin, k, num_cols=part.padded_rows,
                                  options=plan_options)
        # the statistics pair in the first 8 bytes of each block's spare record
        self.stats = native
        words = rb // 4
        self._stats_words_send = self.send_rec.view(torch.int32)[part.max_rows, :2]
        self._stats_all = (self.table_rec.view(torch.int32).view(-1)[part.max_rows * words:],
                           part.world_size, part.block_rows * words)
        self._fwd = fwd or (lambda td, ti, out=None: self.plan.forward(td, ti, out,
                                                                       stats=self._stats_all))
        self._bwd = bwd or (lambda g, ti: self.plan.backward(g, ti, self.grad_table))

    def local_buffers(self):
        """(sp_data, sp_index) strided views [n_local, k] of the send records: write this rank's
        top-k here (``maxk_forward(h, k, out=...)``) and ``gather`` sends them as they are."""
        return self.send_data[: self.n_local], self.send_index[: self.n_local]

    def local_topk(self, h_local: torch.Tensor, mode: str = "exact"):
        """This rank's top-k written straight into its send records, with the fixed-point
        statistics pair fused into the same launch (maxk_topk_cbsr_ex) and written into the
        block's spare record: the NEXT exchange (one only, and only if no torch op has written
        the records since) skips its statistics pass. Returns the ``(sp_data, sp_index)`` views
        of :meth:`local_buffers`."""
        from .ops import maxk_forward
        sd, si = self.local_buffers()
        maxk_forward(h_local, self.dim_k, mode=mode, return_index=True, out=(sd, si),
                     stats=self._stats_words_send if self.stats else None)
        self._stats_version = self.send_rec._version if self.stats else None
        return sd, si

    def _stage(self, sp_data_local: torch.Tensor, sp_index_local: torch.Tensor) -> None:
        n = self.n_local
        fresh = getattr(self, "_stats_version", None)
        if sp_data_local.data_ptr() != self.send_data.data_ptr():
            self.send_data[:n].copy_(sp_data_local)
            fresh = None
        if sp_index_local.data_ptr() != self.send_index.data_ptr():
            self.send_index[:n].copy_(sp_index_local)
            fresh = None
        # this rank's pair, all-gathered with its rows: from the local_topk just before (its
        # records unchanged since: no torch op has bumped their version), else one pass
        self._stats_version = None
        if self.stats and fresh != self.send_rec._version:
            from .ops import cbsr_stats
            cbsr_stats(self.send_data[:n], self.send_index[:n], out=self._stats_words_send)

    def gather(self, sp_data_local: torch.Tensor, sp_index_local: torch.Tensor) -> None:
        """All-gather this rank's CBSR records into the padded table (one RCCL collective)."""
        self._stage(sp_data_local, sp_index_local)
        dist.all_gather_into_tensor(self.table_rec, self.send_rec, group=self.group)

    def forward(self, sp_data_local: torch.Tensor, sp_index_local: torch.Tensor) -> torch.Tensor:
        self.gather(sp_data_local, sp_index_local)
        return self._fwd(self.table_data, self.table_index)

    def compute_forward(self) -> torch.Tensor:
        """The forward's kernels alone on the current table (no exchange): per-rank timing."""
        return self._fwd(self.table_data, self.table_index)

    def backward(self, grad_out_local: torch.Tensor) -> torch.Tensor:
        gp = self._bwd(grad_out_local.contiguous(), self.table_index)
        dist.reduce_scatter_tensor(self.grad_local, gp, op=dist.ReduceOp.SUM, group=self.group)
        return self.grad_local[: self.n_local]

    def compute_backward(self, grad_out_local: torch.Tensor) -> torch.Tensor:
        """The backward's kernels alone (no exchange): per-rank timing."""
        return self._bwd(grad_out_local.contiguous(), self.table_index)

    def unpad_table(self, table: torch.Tensor) -> torch.Tensor:
        """Padded table -> natural node order [N, ...] (tests/inspection)."""
        return torch.cat([table[self.part.table_positions(q, table.device)]
                          for q in range(self.part.world_size)])
