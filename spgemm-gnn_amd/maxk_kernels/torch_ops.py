"""The four reference entry points as registered torch operators (``torch.ops.maxk.*``).

The reference binds its kernels as a pybind11 ``CUDAExtension`` (``/root/reference/setup.py``
lines 23-24): calls are opaque to torch's tracing tools. Here the same four functions are
also registered through ``torch.library`` with shape-only fake kernels, so
``torch.compile(fullgraph=True)``, ``make_fx``/export and FakeTensor shape propagation see
one node per call instead of a graph break, and ``spgemm_forward`` carries its autograd
formula (the SSpMM backward) as a registered derivative.

    torch.ops.maxk.maxk_forward(input, k) -> (sp_data [N, k] f32, sp_index [N, k] u8)
    torch.ops.maxk.maxk_backward(grad_output, indices, dim_origin) -> [N, dim_origin]
    torch.ops.maxk.spgemm_forward(ptr, idx, val, sp_data, sp_index, num_nodes, num_edges,
                                  dim_k, dim_origin) -> out [num_nodes, dim_origin]
    torch.ops.maxk.spgemm_backward(ptr, idx, val, grad_output, sp_index, num_nodes,
                                   num_edges, dim_k, dim_origin) -> grad_sp [num_nodes, dim_k]

The real kernels are :mod:`maxk_kernels.ops` (the HIP C ABI); there is no other
implementation behind these names. Differences from the plain functions, all forced by
the operator schema: ``maxk_forward`` always returns the selectors (the reference drops
them); ``maxk_backward`` takes ``dim_origin`` (a data-dependent width has no fake shape);
``spgemm_forward`` returns ``out`` alone (an operator output may not alias the
``sp_index`` input the reference hands back).
"""
from __future__ import annotations

from typing import Tuple

import torch

from . import ops

_NS = "maxk"


@torch.library.custom_op(f"{_NS}::maxk_forward", mutates_args=())
def maxk_forward(input: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """MaxK top-k -> CBSR (ops.maxk_forward, exact mode)."""
    return ops.maxk_forward(input, k, return_index=True)


@maxk_forward.register_fake
def _(input, k):
    n = input.shape[0]
    return (input.new_empty((n, k)), input.new_empty((n, k), dtype=torch.uint8))


@torch.library.custom_op(f"{_NS}::maxk_backward", mutates_args=())
def maxk_backward(grad_output: torch.Tensor, indices: torch.Tensor,
                  dim_origin: int) -> torch.Tensor:
    """Dense MaxK gradient from the [N, k] CBSR gradient (ops.maxk_backward)."""
    return ops.maxk_backward(grad_output, indices, dim_origin)


@maxk_backward.register_fake
def _(grad_output, indices, dim_origin):
    return grad_output.new_empty((grad_output.shape[0], dim_origin))


@torch.library.custom_op(f"{_NS}::spgemm_forward", mutates_args=())
def spgemm_forward(ptr: torch.Tensor, idx: torch.Tensor, val: torch.Tensor,
                   sp_data: torch.Tensor, sp_index: torch.Tensor, num_nodes: int,
                   num_edges: int, dim_k: int, dim_origin: int) -> torch.Tensor:
    """SpGEMM forward ``out = A @ densify(sp_data, sp_index)`` (ops.spgemm_forward)."""
    return ops.spgemm_forward(ptr, idx, val, sp_data, sp_index, num_nodes, num_edges,
                              dim_k, dim_origin)[0]


@spgemm_forward.register_fake
def _(ptr, idx, val, sp_data, sp_index, num_nodes, num_edges, dim_k, dim_origin):
    return sp_data.new_empty((num_nodes, dim_origin))


@torch.library.custom_op(f"{_NS}::spgemm_backward", mutates_args=())
def spgemm_backward(ptr: torch.Tensor, idx: torch.Tensor, val: torch.Tensor,
                    grad_output: torch.Tensor, sp_index: torch.Tensor, num_nodes: int,
                    num_edges: int, dim_k: int, dim_origin: int) -> torch.Tensor:
    """SSpMM backward ``grad_sp[c, l] = sum_(r,c) val * grad_output[r, sp_index[c, l]]``."""
    return ops.spgemm_backward(ptr, idx, val, grad_output, sp_index, num_nodes, num_edges,
                               dim_k, dim_origin)


@spgemm_backward.register_fake
def _(ptr, idx, val, grad_output, sp_index, num_nodes, num_edges, dim_k, dim_origin):
    return grad_output.new_empty((num_nodes, dim_k))


def _spgemm_setup(ctx, inputs, output):
    ptr, idx, val, _, sp_index, num_nodes, num_edges, dim_k, dim_origin = inputs
    ctx.save_for_backward(ptr, idx, val, sp_index)
    ctx.dims = (num_nodes, num_edges, dim_k, dim_origin)


def _spgemm_backward(ctx, grad):
    ptr, idx, val, sp_index = ctx.saved_tensors
    grad_sp = torch.ops.maxk.spgemm_backward(ptr, idx, val, grad.contiguous(), sp_index,
                                             *ctx.dims)
    return None, None, None, grad_sp, None, None, None, None, None


spgemm_forward.register_autograd(_spgemm_backward, setup_context=_spgemm_setup)


def _maxk_setup(ctx, inputs, output):
    ctx.save_for_backward(output[1])
    ctx.dim_origin = inputs[0].shape[1]


def _maxk_backward(ctx, grad_data, grad_index):
    (sp_index,) = ctx.saved_tensors
    if grad_data is None:
        return None, None
    return torch.ops.maxk.maxk_backward(grad_data.contiguous(), sp_index, ctx.dim_origin), None


maxk_forward.register_autograd(_maxk_backward, setup_context=_maxk_setup)
