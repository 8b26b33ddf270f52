"""autograd surface for the MaxK aggregation path.

The reference has no autograd op pairing ``spgemm_forward`` with ``spgemm_backward``
(the intended pairing is sketched in newmodel.py:60-148 against a
module that does not exist) and its ``MaxKFunction`` (utils/maxk_layers.py:16-45) mixes
``[N, k]`` and dense shapes. Here:

* :class:`MaxKFunction` maps dense ``x [N, D]`` to CBSR ``(sp_data [N, k], sp_index)``;
  its backward is the device scatter ``maxk_backward`` (dense ``[N, D]``), i.e. the
  ``grad * mask`` of utils/models.py:23-26 without materialising the mask.
* :class:`SpGEMMFunction` maps CBSR features to ``Y = A @ densify(sp)`` (SpGEMM forward)
  and back-propagates with the SSpMM kernel, ``grad_sp = (A^T G)`` sampled at the
  selector.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

import torch

from . import ops


@dataclass
class CSRGraph:
    """Destination-row CSR adjacency: row r aggregates from columns idx[ptr[r]:ptr[r+1]].

    This is ``A`` in ``Y = A X``; for DGL's ``update_all(copy_u, ...)`` it is the CSR of
    the in-edges (row = destination node), i.e. ``g.adj_tensors('csc')`` of a DGL graph.
    (The reference takes ``adj_tensors('csr')``, the out-edge CSR, at
    utils/maxk_layers.py:106 — correct only for symmetric graphs; SURVEY §8(b) defect 5.)
    """

    ptr: torch.Tensor
    idx: torch.Tensor
    val: Optional[torch.Tensor] = None
    _values: dict = field(default_factory=dict, repr=False, compare=False)

    def __post_init__(self):
        self.ptr = self.ptr.to(torch.int32).contiguous()
        self.idx = self.idx.to(torch.int32).contiguous()
        if self.val is None:
            self.val = torch.ones(self.idx.numel(), dtype=torch.float32, device=self.idx.device)
        self.val = self.val.to(torch.float32).contiguous()

    @property
    def num_nodes(self) -> int:
        return self.ptr.numel() - 1

    @property
    def num_edges(self) -> int:
        return self.idx.numel()

    @property
    def device(self) -> torch.device:
        return self.ptr.device

    def plan(self, dim_origin: int, dim_k: int) -> ops.GraphPlan:
        return ops.get_plan(self.ptr, self.idx, self.val, self.num_nodes, self.num_edges,
                            dim_origin, dim_k)

    # -- construction -----------------------------------------------------------------
    @classmethod
    def from_edges(cls, src: torch.Tensor, dst: torch.Tensor, num_nodes: int,
                   val: Optional[torch.Tensor] = None) -> "CSRGraph":
        """Edges u -> v (messages flow src -> dst), grouped by destination row."""
        src, dst = src.to(torch.int64), dst.to(torch.int64)
        key = dst * num_nodes + src
        order = torch.argsort(key, stable=True)
        cnt = torch.bincount(dst, minlength=num_nodes)
        ptr = torch.zeros(num_nodes + 1, dtype=torch.int64, device=src.device)
        ptr[1:] = torch.cumsum(cnt, 0)
        return cls(ptr, src[order], None if val is None else val[order])

    @classmethod
    def from_dgl(cls, g) -> "CSRGraph":
        """In-edge CSR of a homogeneous DGL graph (``adj_tensors('csc')``: indptr over
        destinations, indices = sources). Cached on the graph object."""
        cached = getattr(g, "_maxk_csr", None)
        if isinstance(cached, CSRGraph):
            return cached
        indptr, indices, _ = g.adj_tensors("csc")
        csr = cls(indptr, indices)
        try:
            g._maxk_csr = csr
        except AttributeError:  # pragma: no cover - frozen graph objects
            pass
        return csr

    # -- degrees and edge weights -----------------------------------------------------
    def in_degrees(self) -> torch.Tensor:
        return (self.ptr[1:] - self.ptr[:-1]).to(torch.int64)

    def out_degrees(self) -> torch.Tensor:
        return torch.bincount(self.idx.to(torch.int64), minlength=self.num_nodes)

    def edge_values(self, kind: str) -> torch.Tensor:
        """Per-edge weights for the aggregation ``kind`` (cached):

        * ``"sum"`` / ``"none"``: 1
        * ``"mean"`` / ``"right"``: 1 / in_deg(dst)   (DGL fn.mean, GraphConv norm='right')
        * ``"left"``: 1 / out_deg(src)
        * ``"both"``: out_deg(src)^-1/2 * in_deg(dst)^-1/2   (GraphConv norm='both')

        Degrees are clamped to >= 1 (utils/maxk_layers.py:148,302,371).
        """
        v = self._values.get(kind)
        if v is not None:
            return v
        rows = torch.repeat_interleave(torch.arange(self.num_nodes, device=self.device),
                                       self.in_degrees())
        cols = self.idx.to(torch.int64)
        ind = self.in_degrees().clamp(min=1).to(torch.float32)
        outd = self.out_degrees().clamp(min=1).to(torch.float32)
        if kind in ("sum", "none"):
            v = torch.ones(self.num_edges, dtype=torch.float32, device=self.device)
        elif kind in ("mean", "right"):
            v = (1.0 / ind)[rows]
        elif kind == "left":
            v = (1.0 / outd)[cols]
        elif kind == "both":
            v = outd.rsqrt()[cols] * ind.rsqrt()[rows]
        else:
            raise ValueError(f"unknown aggregation weights {kind!r}")
        v = v.contiguous()
        self._values[kind] = v
        return v

    def transposed(self) -> "CSRGraph":
        """A^T with the same edge values (row = source node), cached: the backward of the
        dense aggregation, dX = A^T dY, runs the same SpMM kernel on it."""
        key = ("transposed", self.val.data_ptr(), self.val._version)
        g = self._values.get(key)
        if g is None:
            rows = torch.repeat_interleave(torch.arange(self.num_nodes, device=self.device),
                                           self.in_degrees())
            cols = self.idx.to(torch.int64)
            order = torch.argsort(cols * self.num_nodes + rows, stable=True)
            cnt = torch.bincount(cols, minlength=self.num_nodes)
            ptr = torch.zeros(self.num_nodes + 1, dtype=torch.int64, device=self.device)
            ptr[1:] = torch.cumsum(cnt, 0)
            g = CSRGraph(ptr, rows[order], self.val[order])
            self._values = {k: v for k, v in self._values.items()
                            if not (isinstance(k, tuple) and k[0] == "transposed")}
            self._values[key] = g
        return g

    def with_values(self, kind: str) -> "CSRGraph":
        """Same structure with the ``kind`` edge weights (shares ptr/idx, hence the plan)."""
        key = ("graph", kind)
        g = self._values.get(key)
        if g is None:
            g = CSRGraph(self.ptr, self.idx, self.edge_values(kind))
            self._values[key] = g
        return g


def _mask_padding(grad_data, sp_index, count):
    """ref_compat rows fill ``count`` < k slots; the padding slots (0.0f, 0) carry no gradient:
    each is pointed at the row's last filled slot with that slot's gradient, so the scatter
    (last slot wins) never writes into a feature 0 that was not selected."""
    count = count.to(torch.int64)
    k = sp_index.shape[1]
    pad = torch.arange(k, device=count.device)[None, :] >= count[:, None]
    last = (count - 1).clamp(min=0)[:, None]
    g_last = torch.where(count[:, None] > 0, grad_data.gather(1, last),
                         torch.zeros_like(grad_data[:, :1]))
    sp_index = torch.where(pad, sp_index.gather(1, last), sp_index).contiguous()
    grad_data = torch.where(pad, g_last, grad_data).contiguous()
    return grad_data, sp_index


class MaxKFunction(torch.autograd.Function):
    """x [N, D] -> CBSR (sp_data, sp_index); backward = the device scatter of grad_data
    into the selected features (the ``grad * mask`` of utils/models.py:23-26).

    ref_compat mode can fill fewer than k slots; the reference pads them with (0.0f, 0)
    (SURVEY §8 a1). Those slots pass no gradient: before the scatter (last slot wins) each
    padding slot is pointed at the row's last filled slot with that slot's gradient, so a
    padding slot never writes (A^T G)[c, 0] into a feature 0 that was not selected."""

    @staticmethod
    def forward(ctx, x: torch.Tensor, k: int, mode: str = "exact"):
        x = x.contiguous()
        if mode == "exact":
            sp_data, sp_index = ops.maxk_forward(x, k, mode=mode, return_index=True)
            ctx.save_for_backward(sp_index)
        else:
            sp_data, sp_index, count = ops.maxk_forward(x, k, mode=mode, return_index=True,
                                                        return_count=True)
            ctx.save_for_backward(sp_index, count)
        ctx.dim_origin = x.shape[1]
        ctx.mark_non_differentiable(sp_index)
        return sp_data, sp_index

    @staticmethod
    def backward(ctx, grad_data, grad_index):
        saved = ctx.saved_tensors
        sp_index = saved[0]
        grad_data = grad_data.contiguous()
        if len(saved) == 2:
            grad_data, sp_index = _mask_padding(grad_data, sp_index, saved[1])
        grad_x = ops.maxk_backward(grad_data, sp_index, dim_origin=ctx.dim_origin)
        return grad_x, None, None


class SpGEMMFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, sp_data: torch.Tensor, sp_index: torch.Tensor, graph: CSRGraph,
                dim_origin: int):
        k = sp_data.shape[1]
        plan = graph.plan(dim_origin, k)
        out, _ = ops.spgemm_forward(graph.ptr, graph.idx, graph.val, sp_data.contiguous(),
                                    sp_index, graph.num_nodes, graph.num_edges, k,
                                    dim_origin, plan=plan)
        ctx.save_for_backward(sp_index)
        ctx.graph = graph
        ctx.plan = plan  # the backward uses the same plan (no cache lookup, no rebuild)
        ctx.dims = (dim_origin, k)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        (sp_index,) = ctx.saved_tensors
        graph = ctx.graph
        dim_origin, k = ctx.dims
        grad_sp = None
        if ctx.needs_input_grad[0]:
            grad_sp = ops.spgemm_backward(graph.ptr, graph.idx, graph.val,
                                          grad_out.contiguous(), sp_index, graph.num_nodes,
                                          graph.num_edges, k, dim_origin, plan=ctx.plan)
        return grad_sp, None, None, None


class DenseAggFunction(torch.autograd.Function):
    """Y = A X on dense features (DGL ``update_all(copy_u('h'), sum)`` with the graph's edge
    values, i.e. mean / GraphConv normalisation through ``CSRGraph.with_values``): the
    aggregation of the ReLU layers (utils/models.py:140,252 with ``--nonlinear relu``).
    Forward and backward both run ``maxk_dense_spmm_csr``; the backward on A^T."""

    @staticmethod
    def forward(ctx, x: torch.Tensor, graph: CSRGraph):
        ctx.graph = graph
        return ops.dense_spmm(graph.ptr, graph.idx, graph.val, x.contiguous())

    @staticmethod
    def backward(ctx, grad_out):
        grad_x = None
        if ctx.needs_input_grad[0]:
            gt = ctx.graph.transposed()
            grad_x = ops.dense_spmm(gt.ptr, gt.idx, gt.val, grad_out.contiguous())
        return grad_x, None


class MaxKAggregateFunction(torch.autograd.Function):
    """``A @ densify(MaxK(x))`` as one producer-consumer pair (utils/maxk_layers.py:16-34:
    MaxK feeding the SpGEMM). The top-k writes the CBSR features straight into the layout
    the plan's forward gathers (its packed records when ``fwd_layout`` is 1, GraphPlan.new_cbsr)
    together with the fixed-point statistics of the emitted rows (maxk_topk_cbsr_ex), so the
    forward launches no per-call pack or statistics pass. Backward: the SSpMM on the same plan
    (selectors read at the record stride), then the MaxK scatter (same rules as MaxKFunction
    for ref_compat padding)."""

    @staticmethod
    def forward(ctx, x: torch.Tensor, graph: CSRGraph, k: int, mode: str = "exact"):
        x = x.contiguous()
        d = x.shape[1]
        plan = graph.plan(d, k)
        sp_data, sp_index = plan.new_cbsr()
        stats = torch.empty(2, dtype=torch.int32, device=x.device)
        res = ops.maxk_forward(x, k, mode=mode, return_index=True, out=(sp_data, sp_index),
                               stats=stats, return_count=mode != "exact")
        out = plan.forward(sp_data, sp_index, stats=stats.view(1, 2))
        ctx.save_for_backward(sp_index, *res[2:])
        ctx.plan = plan
        ctx.dim_origin = d
        return out

    @staticmethod
    def backward(ctx, grad_out):
        saved = ctx.saved_tensors
        sp_index = saved[0]
        grad_x = None
        if ctx.needs_input_grad[0]:
            grad_sp = ctx.plan.backward(grad_out.contiguous(), sp_index)
            if len(saved) == 2:
                grad_sp, sp_index = _mask_padding(grad_sp, sp_index, saved[1])
            grad_x = ops.maxk_backward(grad_sp, sp_index, dim_origin=ctx.dim_origin)
        return grad_x, None, None, None


def dense_aggregate(x: torch.Tensor, graph: CSRGraph) -> torch.Tensor:
    """Y = A @ x for dense x (ReLU layers), differentiable in x."""
    return DenseAggFunction.apply(x, graph)


def densify(sp_data: torch.Tensor, sp_index: torch.Tensor, dim_origin: int) -> torch.Tensor:
    """Dense ``[N, D]`` view of CBSR features (differentiable in sp_data; duplicate
    selectors sum, as in the kernels)."""
    out = torch.zeros((sp_data.shape[0], dim_origin), dtype=sp_data.dtype,
                      device=sp_data.device)
    return out.scatter_add(1, sp_index.long(), sp_data)


def maxk(x: torch.Tensor, k: int, mode: str = "exact"):
    """(sp_data, sp_index) = MaxK(x), differentiable in x."""
    return MaxKFunction.apply(x, k, mode)


def spgemm(sp_data: torch.Tensor, sp_index: torch.Tensor, graph: CSRGraph,
           dim_origin: int) -> torch.Tensor:
    """Y = A @ densify(sp_data, sp_index), differentiable in sp_data."""
    return SpGEMMFunction.apply(sp_data, sp_index, graph, dim_origin)


def maxk_aggregate(x: torch.Tensor, graph: CSRGraph, k: int, mode: str = "exact",
                   ) -> torch.Tensor:
    """Fused MaxK + aggregation: ``A @ (x * topk_mask(x))`` (DGL: MaxK.apply then
    update_all(u_mul_e, sum) with edge weights ``graph.val``), differentiable in x; the
    top-k hands the forward its records and statistics (MaxKAggregateFunction)."""
    return MaxKAggregateFunction.apply(x, graph, k, mode)
