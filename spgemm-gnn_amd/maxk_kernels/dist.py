"""Row-partitioned MaxK aggregation over several GPUs of one node (one process per GPU).

The reference is single-GPU (no NCCL / torch.distributed anywhere; multi-GPU is future
work in README_INTEGRATED.md:382). The path shards by destination rows with one real
exchange per direction:

* partition: contiguous row ranges balanced by nnz; rank q owns rows [start_q, end_q),
  their CSR slice (columns keep pointing at any node) and computes the top-k of its own
  rows (weights are replicated);
* forward : RCCL all-gathers of the k-sparse CBSR block (sp_data f32 and sp_index u8)
  straight into the tables the kernels read; the rank's top-k can be written directly into
  its send buffers (``local_buffers``), so the exchange moves no extra copies. Then the
  local SpGEMM over the rank's rows with rectangular plans whose column ids are remapped
  into the gathered table (once, at partition time);
* backward: the local SSpMM produces a partial grad_sp for every (padded) column; an
  RCCL reduce-scatter (sum) returns each rank its own rows' gradient.

Fixed-point statistics: with one phase, every rank's block of the table ends in a spare row.
Before the all-gather the rank writes the fixed-point statistics of its own rows into the
selector bytes of that row (``maxk_cbsr_stats``: two words; the value row stays zero, so the
row adds nothing anywhere), the gathered index table carries one pair per rank and the
forward reads those W pairs (``maxk_spgemm_forward_ex``) instead of scanning the whole table.

Local-columns-first split (``split=True``, one phase, forward only): the rank's edges are
cut into those whose column it owns and the rest, with a plan each. The forward runs the
local plan on the send buffers while the all-gather is in flight, then the remote plan
accumulates on the gathered table. The backward runs one plan over all the rank's edges and
then the reduce-scatter: splitting it too (remote plan, reduce-scatter in flight while the
local plan runs) cost more than the exchange it hides (Reddit k=16, one rank of W=2 / 8:
0.88 -> 1.34 ms / 0.23 -> 0.32 ms, ``tools/shard_time.py``), since each part's column
blocks see half as many edges per grad_out row.

Column phases (``phases`` P > 1): every rank's rows are cut into P parts and the table is
laid out phase-major (phase p holds part p of every rank), so each phase is one all-gather
and one reduce-scatter of its own. The rank keeps one plan per phase (its edges split by the
phase of their column). The all-gather of phase p+1 then runs while the SpGEMM of phase p
(accumulating into the same output) computes, and the reduce-scatter of phase p while the
SSpMM of phase p+1 computes. P = 1 is the plain one-shot exchange.

Bytes exchanged per step are 5kN (all-gathers) + 4kN (reduce-scatter), i.e. 18.6 MB +
14.9 MB for Reddit at k=16, against 238 MB for all-gathering dense features.
"""
from __future__ import annotations

from typing import Callable, List, Optional

import torch
import torch.distributed as dist


class RowPartition:
    """Contiguous destination-row ranges with ~equal nnz per rank, and the phase-major
    layout of the all-gathered CBSR table (``phases`` parts per rank; with one phase each
    rank's block ends in a spare row that carries its fixed-point statistics)."""

    def __init__(self, ptr: torch.Tensor, world_size: int, phases: int = 1,
                 stats_row: Optional[bool] = None):
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
        self.phases = max(1, int(phases))
        self.stats_row = (self.phases == 1) if stats_row is None else bool(stats_row)
        if self.stats_row and self.phases != 1:
            raise ValueError("the statistics row needs a one-phase partition")
        self.rows_per_phase = -(-self.max_rows // self.phases)  # node rows of a rank per phase
        self.phase_rows = self.rows_per_phase + (1 if self.stats_row else 0)
        self.phase_cols = w * self.phase_rows                  # table rows of one phase
        self.send_rows = self.phases * self.phase_rows         # >= max_rows
        self.padded_rows = self.phases * self.phase_cols

    def rows(self, rank: int):
        return int(self.bounds[rank]), int(self.bounds[rank + 1])

    def _position(self, q: torch.Tensor, off: torch.Tensor) -> torch.Tensor:
        ph = off // self.rows_per_phase
        return ph * self.phase_cols + q * self.phase_rows + (off - ph * self.rows_per_phase)

    def remap_columns(self, idx: torch.Tensor) -> torch.Tensor:
        """Global column id -> position in the padded (phase-major) all-gather table."""
        b = self.bounds.to(idx.device)
        c = idx.to(torch.int64)
        q = torch.searchsorted(b, c, right=True) - 1
        return self._position(q, c - b[q]).to(torch.int32)

    def table_positions(self, rank: int, device=None) -> torch.Tensor:
        """Table rows holding rank's nodes, in node order (int64 [n_rank])."""
        a, b = self.rows(rank)
        off = torch.arange(b - a, dtype=torch.int64, device=device)
        return self._position(torch.full_like(off, rank), off)

    def stats_position(self, rank: int) -> int:
        """Table row of rank's statistics pair (one-phase partitions)."""
        return rank * self.phase_rows + self.rows_per_phase

    def local_csr(self, ptr: torch.Tensor, idx: torch.Tensor, val: torch.Tensor, rank: int):
        """(ptr, remapped idx, val) of rank's rows; ptr rebased to 0."""
        r0, r1 = self.rows(rank)
        e0, e1 = int(ptr[r0]), int(ptr[r1])
        lptr = (ptr[r0:r1 + 1].to(torch.int64) - e0).to(torch.int32).contiguous()
        lidx = self.remap_columns(idx[e0:e1]).contiguous()
        lval = val[e0:e1].contiguous()
        return lptr, lidx, lval

    def phase_csr(self, lptr: torch.Tensor, lidx: torch.Tensor, lval: torch.Tensor, phase: int):
        """The edges of a local CSR (remapped columns) whose column lies in ``phase``, with
        columns rebased to that phase's table block [0, phase_cols)."""
        lo = phase * self.phase_cols
        return select_csr(lptr, lidx, lval, (lidx >= lo) & (lidx < lo + self.phase_cols), lo)


def select_csr(lptr: torch.Tensor, lidx: torch.Tensor, lval: torch.Tensor,
               keep: torch.Tensor, shift: int = 0):
    """The edges of a CSR where ``keep`` holds (row order kept), columns minus ``shift``."""
    n = lptr.numel() - 1
    rows = torch.repeat_interleave(torch.arange(n, device=lptr.device),
                                   (lptr[1:] - lptr[:-1]).to(torch.int64))
    cnt = torch.bincount(rows[keep], minlength=n)
    pptr = torch.zeros(n + 1, dtype=torch.int64, device=lptr.device)
    pptr[1:] = torch.cumsum(cnt, 0)
    return (pptr.to(torch.int32).contiguous(), (lidx[keep] - shift).to(torch.int32).contiguous(),
            lval[keep].contiguous())


# injected per-part compute (CPU tests): fwd(part, table_data, table_index, out) -> out (out
# is None for the first part, else the output to accumulate into); bwd(part, grad_out,
# table_index) -> the part's grad rows. A part reads the table given by ShardedAggregation
# (its phase's block, or for the split: the send buffers / the whole table).
FwdFn = Callable[[int, torch.Tensor, torch.Tensor, Optional[torch.Tensor]], torch.Tensor]
BwdFn = Callable[[int, torch.Tensor, torch.Tensor], torch.Tensor]


class ShardedAggregation:
    """One rank's share of Y = A densify(sp) and of its SSpMM backward.

    ``fwd``/``bwd`` default to the gfx950 kernels through one rectangular GraphPlan per
    part (``plan_options``: the same knobs as ``GraphPlan(options=...)``, e.g.
    ``{"bwd_algo": 3}``); tests on CPU (gloo) inject checker callables to exercise the
    partition, the layouts and the collectives. ``parts[i]`` = (ptr, idx, val, num_cols) of
    part i: the column phases, or (split) the own-column and the remote-column edges.
    """

    def __init__(self, part: RowPartition, rank: int, ptr: torch.Tensor, idx: torch.Tensor,
                 val: torch.Tensor, dim_origin: int, dim_k: int,
                 group: Optional[dist.ProcessGroup] = None, fwd: Optional[FwdFn] = None,
                 bwd: Optional[BwdFn] = None, plan_options: Optional[dict] = None,
                 split: bool = False):
        self.part, self.rank, self.group = part, rank, group
        self.dim_origin, self.dim_k = int(dim_origin), int(dim_k)
        self.r0, self.r1 = part.rows(rank)
        self.n_local = self.r1 - self.r0
        self.ptr, self.idx, self.val = part.local_csr(ptr, idx, val, rank)
        dev = self.ptr.device
        P, k = part.phases, self.dim_k
        if split and P != 1:
            raise ValueError("the local-columns-first split needs a one-phase partition")
        self.split = bool(split)
        # padded send buffers (rows >= n_local stay zero) and the all-gathered tables
        self.send_data = torch.zeros((part.send_rows, k), dtype=torch.float32, device=dev)
        self.send_index = torch.zeros((part.send_rows, k), dtype=torch.uint8, device=dev)
        self.table_data = torch.empty((part.padded_rows, k), dtype=torch.float32, device=dev)
        self.table_index = torch.empty((part.padded_rows, k), dtype=torch.uint8, device=dev)
        self.grad_table = torch.empty((part.padded_rows, k), dtype=torch.float32, device=dev)
        self.grad_local = torch.empty((part.send_rows, k), dtype=torch.float32, device=dev)
        if self.split:
            lo = rank * part.phase_rows
            own = (self.idx >= lo) & (self.idx < lo + self.n_local)
            # own columns, remote columns (forward), all edges (backward)
            self.parts = [select_csr(self.ptr, self.idx, self.val, own, lo) + (max(1, self.n_local),),
                          select_csr(self.ptr, self.idx, self.val, ~own) + (part.padded_rows,),
                          (self.ptr, self.idx, self.val, part.padded_rows)]
        else:
            self.parts = [part.phase_csr(self.ptr, self.idx, self.val, p) + (part.phase_cols,)
                          for p in range(P)]
        self.plans: List = []
        native = fwd is None or bwd is None
        if native:
            from .ops import GraphPlan
            for pp, pi, pv, nc in self.parts:
                self.plans.append(GraphPlan(pp, pi, pv, self.n_local, pi.numel(),
                                            self.dim_origin, self.dim_k, num_cols=nc,
                                            options=plan_options))
        # the statistics pair in the selector bytes of the send buffer's spare row (one
        # phase, native kernels; 4-byte aligned words: k % 4 == 0, k >= 8)
        self.stats = native and part.stats_row and k % 4 == 0 and k >= 8
        rp = part.rows_per_phase
        self._stats_local = (self._words(self.send_index, rp), 1, 2) if self.stats else None
        self._stats_all = ((self._words(self.table_index, rp), part.world_size,
                            part.phase_rows * k // 4) if self.stats else None)
        self._fwd = fwd or self._native_fwd
        self._bwd = bwd or (lambda i, g, ti: self.plans[i].backward(g, ti, self._grad_dst(i)))

    @staticmethod
    def _words(index_table: torch.Tensor, row: int) -> torch.Tensor:
        """int32 view of a u8 table from ``row`` on (the statistics words of a spare row)."""
        return index_table[row:].view(-1).view(torch.int32)

    def _native_fwd(self, i, td, ti, out):
        stats = None
        if self.stats:
            stats = self._stats_local if (self.split and i == 0) else self._stats_all
        return self.plans[i].forward(td, ti, out, accumulate=out is not None, stats=stats)

    def _grad_dst(self, i):
        if self.split:
            return self.grad_table
        return self._slice(self.grad_table, i)

    @property
    def plan(self):
        """The plan of a one-part partition (bench.py's per-kernel timing)."""
        return self.plans[0] if len(self.plans) == 1 else None

    def _slice(self, table: torch.Tensor, p: int) -> torch.Tensor:
        c = self.part.phase_cols
        return table[p * c: (p + 1) * c]

    def _send_slice(self, buf: torch.Tensor, p: int) -> torch.Tensor:
        r = self.part.phase_rows
        return buf[p * r: (p + 1) * r]

    def local_buffers(self):
        """(sp_data, sp_index) views [n_local, k] of the send buffers: write this rank's
        top-k here (``maxk_forward(h, k, out=...)``) and ``gather`` sends them as they are."""
        return self.send_data[: self.n_local], self.send_index[: self.n_local]

    def _stage(self, sp_data_local: torch.Tensor, sp_index_local: torch.Tensor) -> None:
        n = self.n_local
        if sp_data_local.data_ptr() != self.send_data.data_ptr():
            self.send_data[:n].copy_(sp_data_local)
        if sp_index_local.data_ptr() != self.send_index.data_ptr():
            self.send_index[:n].copy_(sp_index_local)
        if self.stats:  # this rank's pair, all-gathered with its rows
            from .ops import cbsr_stats
            cbsr_stats(self.send_data[:n], self.send_index[:n],
                       out=self.stats_words(self.send_index, self.part.rows_per_phase))

    @staticmethod
    def stats_words(index_table: torch.Tensor, row: int) -> torch.Tensor:
        """The 2 int32 statistics words in the selector bytes of a spare row."""
        return index_table[row].view(torch.int32)[:2]

    def _gather_phase(self, p: int, async_op: bool):
        w1 = dist.all_gather_into_tensor(self._slice(self.table_data, p),
                                         self._send_slice(self.send_data, p),
                                         group=self.group, async_op=async_op)
        w2 = dist.all_gather_into_tensor(self._slice(self.table_index, p),
                                         self._send_slice(self.send_index, p),
                                         group=self.group, async_op=async_op)
        return (w1, w2)

    def gather(self, sp_data_local: torch.Tensor, sp_index_local: torch.Tensor) -> None:
        """All-gather this rank's CBSR rows into the padded tables (RCCL over xGMI)."""
        self._stage(sp_data_local, sp_index_local)
        for p in range(self.part.phases):
            self._gather_phase(p, async_op=False)

    def forward(self, sp_data_local: torch.Tensor, sp_index_local: torch.Tensor) -> torch.Tensor:
        self._stage(sp_data_local, sp_index_local)
        P = self.part.phases
        works = [self._gather_phase(p, async_op=True) for p in range(P)]
        if self.split:
            # own columns from the send buffers while the exchange is in flight
            out = self._fwd(0, self.send_data[: self.n_local], self.send_index[: self.n_local],
                            None)
            for wk in works[0]:
                wk.wait()
            return self._fwd(1, self.table_data, self.table_index, out)
        out = None
        for p in range(P):
            for wk in works[p]:
                wk.wait()   # the compute stream waits for phase p only
            out = self._fwd(p, self._slice(self.table_data, p), self._slice(self.table_index, p),
                            out)
        return out

    def compute_forward(self) -> torch.Tensor:
        """The forward's kernels alone on the current tables (no exchange): per-rank timing."""
        if self.split:
            out = self._fwd(0, self.send_data[: self.n_local], self.send_index[: self.n_local],
                            None)
            return self._fwd(1, self.table_data, self.table_index, out)
        out = None
        for p in range(self.part.phases):
            out = self._fwd(p, self._slice(self.table_data, p), self._slice(self.table_index, p),
                            out)
        return out

    def backward(self, grad_out_local: torch.Tensor) -> torch.Tensor:
        g = grad_out_local.contiguous()
        if self.split:  # the all-edges plan, then the one-shot reduce-scatter
            gp = self._bwd(2, g, self.table_index)
            dist.reduce_scatter_tensor(self.grad_local, gp, op=dist.ReduceOp.SUM,
                                       group=self.group)
            return self.grad_local[: self.n_local]
        works = []
        for p in range(self.part.phases):
            gp = self._bwd(p, g, self._slice(self.table_index, p))
            works.append(dist.reduce_scatter_tensor(self._send_slice(self.grad_local, p), gp,
                                                    op=dist.ReduceOp.SUM, group=self.group,
                                                    async_op=True))
        for wk in works:
            wk.wait()
        return self.grad_local[: self.n_local]

    def compute_backward(self, grad_out_local: torch.Tensor) -> None:
        """The backward's kernels alone (no exchange): per-rank timing."""
        g = grad_out_local.contiguous()
        if self.split:
            self._bwd(2, g, self.table_index)
            return
        for p in range(self.part.phases):
            self._bwd(p, g, self._slice(self.table_index, p))

    def unpad_table(self, table: torch.Tensor) -> torch.Tensor:
        """Padded phase-major table -> natural node order [N, ...] (tests/inspection)."""
        return torch.cat([table[self.part.table_positions(q, table.device)]
                          for q in range(self.part.world_size)])
