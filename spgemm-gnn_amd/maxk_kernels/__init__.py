"""maxk_kernels — MI355X-native drop-in for the reference's ``maxk_kernels`` extension.

``import maxk_kernels`` exposes the reference's four bound functions with the same
positional signatures:

    maxk_forward(input, k) -> sp_data [N, k]
    maxk_backward(grad_output, indices) -> [N, D]
    spgemm_forward(ptr, idx, val, sp_data, sp_index, num_nodes, num_edges, dim_k, dim_origin)
        -> (out [N, D], sp_index)
    spgemm_backward(ptr, idx, val, grad_output, sp_index, num_nodes, num_edges, dim_k,
                    dim_origin) -> grad_sp [N, k]

all running hand-written gfx950 HIP kernels through the C ABI of include/maxk_hip.h
(libmaxk_hip.so). There is no fallback: if the library is missing the import fails.
"""
from ._lib import LIB_PATH, MaxKError, lib  # noqa: F401  (loads libmaxk_hip.so)
from .ops import (  # noqa: F401
    TOPK_MODES,
    GraphPlan,
    cbsr_stats,
    clear_plan_cache,
    dense_spmm,
    get_plan,
    maxk_backward,
    maxk_forward,
    plan_col_order,
    spgemm_backward,
    spgemm_forward,
)
from .autograd import (  # noqa: F401
    CSRGraph,
    DenseAggFunction,
    MaxKAggregateFunction,
    MaxKFunction,
    SpGEMMFunction,
    dense_aggregate,
    densify,
    maxk,
    maxk_aggregate,
    spgemm,
)

from . import torch_ops  # noqa: F401,E402  (registers torch.ops.maxk.*)
from .layers import (  # noqa: F401,E402
    MaxKGCN,
    MaxKGCNConv,
    MaxKGIN,
    MaxKGINConv,
    MaxKSAGE,
    MaxKSAGEConv,
)

__all__ = [
    "maxk_forward", "maxk_backward", "spgemm_forward", "spgemm_backward",
    "dense_spmm", "cbsr_stats", "plan_col_order", "GraphPlan", "get_plan", "clear_plan_cache", "CSRGraph",
    "MaxKFunction", "MaxKAggregateFunction", "SpGEMMFunction", "maxk", "spgemm", "maxk_aggregate", "MaxKError",
    "densify", "MaxKSAGEConv", "MaxKGCNConv", "MaxKGINConv", "MaxKSAGE", "MaxKGCN",
    "MaxKGIN", "dense_aggregate", "DenseAggFunction",
]

ABI_VERSION = lib.maxk_abi_version()
