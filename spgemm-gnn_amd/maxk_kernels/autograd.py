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

from dataclasses import dataclass
from typing import Optional

import torch

from . import ops


@dataclass
class CSRGraph:
    """Destination-row CSR adjacency: row r aggregates from columns idx[ptr[r]:ptr[r+1]].

    This is ``A`` in ``Y = A X``; for DGL's ``update_all(copy_u, ...)`` it is the CSR of
    the in-edges (row = destination node), i.e. ``g.adj_tensors('csc')`` of a DGL graph.
    """

    ptr: torch.Tensor
    idx: torch.Tensor
    val: torch.Tensor

    @property
    def num_nodes(self) -> int:
        return self.ptr.numel() - 1

    @property
    def num_edges(self) -> int:
        return self.idx.numel()

    def plan(self, dim_origin: int, dim_k: int) -> ops.GraphPlan:
        return ops.get_plan(self.ptr, self.idx, self.val, self.num_nodes, self.num_edges,
                            dim_origin, dim_k)


class MaxKFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, k: int, mode: str = "exact"):
        x = x.contiguous()
        sp_data, sp_index = ops.maxk_forward(x, k, mode=mode, return_index=True)
        ctx.save_for_backward(sp_index)
        ctx.dim_origin = x.shape[1]
        ctx.mark_non_differentiable(sp_index)
        return sp_data, sp_index

    @staticmethod
    def backward(ctx, grad_data, grad_index):
        (sp_index,) = ctx.saved_tensors
        grad_x = ops.maxk_backward(grad_data.contiguous(), sp_index, dim_origin=ctx.dim_origin)
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
                                          graph.num_edges, k, dim_origin,
                                          plan=graph.plan(dim_origin, k))
        return grad_sp, None, None, None


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
    update_all(u_mul_e, sum) with edge weights ``graph.val``)."""
    sp_data, sp_index = maxk(x, k, mode)
    return spgemm(sp_data, sp_index, graph, x.shape[1])
