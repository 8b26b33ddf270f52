"""Drop-in MaxK graph layers on the gfx950 SpGEMM / SSpMM kernels.

Replaces the reference's ``MaxKSAGEConv`` (utils/maxk_layers.py:47-265) and
``MaxKGCNConv`` (utils/maxk_layers.py:267-448) with the same constructor signatures, and
``MaxKSAGE`` / ``MaxKGCN`` (utils/integrated_models.py:8-143) with the same structure,
but with the SURVEY §8(b) caller defects fixed:

* MaxK yields CBSR ``(sp_data, sp_index)`` directly; no dense ``[N, k]`` misuse, no
  per-row Python ``_extract_sparse_format`` loop, no uint8 wrap (D <= 256 is checked);
* the aggregation runs over the in-edge CSR (destination rows) and is differentiable:
  SpGEMM forward, SSpMM backward, MaxK backward scatter;
* edge weights are built on the device once per graph (no per-row ``.item()`` loop).

Numerics follow DGL on the same MaxK input (the semantics the reference trained with,
utils/models.py:12-26 + dglnn.SAGEConv / dglnn.GraphConv):

* ``MaxKSAGEConv``: ``rst = fc_self(x) + fc_neigh(mean_{u->v} x_u) (+ bias)``, then
  ``norm``; ``x = feat_drop(MaxK(feat))``. Dropout acts on the k kept values only (the
  other entries are zero either way). The reference's layer applies MaxK after
  ``fc_neigh`` and dropout to its output (maxk_layers.py:85-88,183); ``maxk_after_fc=True``
  keeps that ordering.
* ``MaxKGCNConv``: ``rst = A_norm MaxK(feat W) (+ bias)`` with ``A_norm`` the GraphConv
  normalisation ('both', 'right', 'left', 'none'); with ``weight=False`` this is
  ``dglnn.GraphConv(weight=None)`` applied to ``MaxK(feat)``.

``graph`` may be a :class:`~maxk_kernels.autograd.CSRGraph` or a DGL graph (converted
with ``adj_tensors('csc')`` when DGL is installed; it is not required).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .autograd import CSRGraph, densify, maxk, spgemm


def as_csr(graph) -> CSRGraph:
    if isinstance(graph, CSRGraph):
        return graph
    if hasattr(graph, "adj_tensors"):
        return CSRGraph.from_dgl(graph)
    raise TypeError("graph must be a maxk_kernels.CSRGraph or a DGL graph")


def _sparse_dropout(sp_data: torch.Tensor, p: float, training: bool) -> torch.Tensor:
    return F.dropout(sp_data, p, training) if p > 0 else sp_data


class MaxKSAGEConv(nn.Module):
    """GraphSAGE layer with MaxK sparsity and the fused aggregation kernels.

    Signature of utils/maxk_layers.py:51-52 plus ``bias`` (dglnn.SAGEConv has one) and
    ``maxk_after_fc`` (the reference layer's MaxK placement).
    """

    def __init__(self, in_feats, out_feats, aggregator_type="mean", feat_drop=0., norm=None,
                 maxk=32, bias=True, maxk_after_fc=False, topk_mode="exact"):
        super().__init__()
        if aggregator_type not in ("mean", "sum"):
            raise ValueError(f"Unsupported aggregator type: {aggregator_type}")
        self.in_feats = in_feats
        self.out_feats = out_feats
        self.aggregator_type = aggregator_type
        self.maxk = maxk
        self.maxk_after_fc = maxk_after_fc
        self.topk_mode = topk_mode
        self.fc_self = nn.Linear(in_feats, out_feats, bias=False)
        self.fc_neigh = nn.Linear(in_feats, out_feats, bias=False)
        self.bias = nn.Parameter(torch.zeros(out_feats)) if bias else None
        self.norm = norm
        self.feat_drop = float(feat_drop)
        self.reset_parameters()

    def reset_parameters(self):
        gain = nn.init.calculate_gain("relu")
        nn.init.xavier_uniform_(self.fc_self.weight, gain=gain)
        nn.init.xavier_uniform_(self.fc_neigh.weight, gain=gain)
        if self.bias is not None:
            nn.init.zeros_(self.bias)

    def forward(self, graph, feat: torch.Tensor) -> torch.Tensor:
        csr = as_csr(graph).with_values(self.aggregator_type)
        if self.maxk_after_fc:
            # reference ordering (maxk_layers.py:85-88): MaxK(fc_neigh(feat)) aggregated
            h_self = self.fc_self(feat)
            sp_data, sp_index = maxk(self.fc_neigh(feat), self.maxk, self.topk_mode)
            sp_data = _sparse_dropout(sp_data, self.feat_drop, self.training)
            rst = h_self + spgemm(sp_data, sp_index, csr, self.out_feats)
        else:
            sp_data, sp_index = maxk(feat, self.maxk, self.topk_mode)
            sp_data = _sparse_dropout(sp_data, self.feat_drop, self.training)
            x = densify(sp_data, sp_index, self.in_feats)
            neigh = spgemm(sp_data, sp_index, csr, self.in_feats)
            rst = self.fc_self(x) + self.fc_neigh(neigh)
        if self.bias is not None:
            rst = rst + self.bias
        if self.norm is not None:
            rst = self.norm(rst)
        return rst


class MaxKGCNConv(nn.Module):
    """GCN layer with MaxK sparsity (signature of utils/maxk_layers.py:271-272, plus
    ``feat_drop``: dropout between MaxK and the aggregation, as utils/models.py:262-264)."""

    def __init__(self, in_feats, out_feats, norm="both", weight=True, bias=True,
                 allow_zero_in_degree=False, maxk=32, topk_mode="exact", feat_drop=0.):
        super().__init__()
        if norm not in ("both", "right", "left", "none"):
            raise ValueError(f"Invalid norm value {norm!r}")
        self.in_feats = in_feats
        self.out_feats = out_feats
        self.norm = norm
        self.maxk = maxk
        self.topk_mode = topk_mode
        self.allow_zero_in_degree = allow_zero_in_degree
        self.feat_drop = float(feat_drop)
        self.weight = nn.Parameter(torch.empty(in_feats, out_feats)) if weight else None
        self.bias = nn.Parameter(torch.empty(out_feats)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        if self.weight is not None:
            nn.init.xavier_uniform_(self.weight)
        if self.bias is not None:
            nn.init.zeros_(self.bias)

    def forward(self, graph, feat: torch.Tensor) -> torch.Tensor:
        csr = as_csr(graph)
        if not self.allow_zero_in_degree and bool((csr.in_degrees() == 0).any()):
            raise ValueError("Graph has nodes with zero in-degree")
        if self.weight is not None:
            feat = feat @ self.weight
        sp_data, sp_index = maxk(feat, self.maxk, self.topk_mode)
        sp_data = _sparse_dropout(sp_data, self.feat_drop, self.training)
        rst = spgemm(sp_data, sp_index, csr.with_values(self.norm), feat.shape[1])
        if self.bias is not None:
            rst = rst + self.bias
        return rst


class MaxKSAGE(nn.Module):
    """utils/integrated_models.py:8-66 (MaxK applied inside each MaxKSAGEConv)."""

    def __init__(self, in_size, hid_size, num_hid_layers, out_size, maxk=32, feat_drop=0.5,
                 norm=False, nonlinear="maxk"):
        super().__init__()
        if nonlinear != "maxk":
            raise ValueError("only nonlinear='maxk' runs on the MaxK kernels")
        self.lin_in = nn.Linear(in_size, hid_size)
        self.lin_out = nn.Linear(hid_size, out_size)
        self.layers = nn.ModuleList(
            MaxKSAGEConv(hid_size, hid_size, "mean", feat_drop=feat_drop,
                         norm=nn.LayerNorm(hid_size) if norm else None, maxk=maxk)
            for _ in range(num_hid_layers))
        nn.init.xavier_uniform_(self.lin_in.weight)
        nn.init.xavier_uniform_(self.lin_out.weight)

    def forward(self, g, x):
        x = self.lin_in(x)
        for layer in self.layers:
            x = layer(g, x)
        return self.lin_out(x)


class MaxKGCN(nn.Module):
    """utils/models.py:232-270 GCN (lin -> MaxK -> dropout -> GraphConv(weight=None))."""

    def __init__(self, in_size, hid_size, num_hid_layers, out_size, maxk=32, feat_drop=0.5,
                 norm=False, nonlinear="maxk"):
        super().__init__()
        if nonlinear != "maxk":
            raise ValueError("only nonlinear='maxk' runs on the MaxK kernels")
        self.lin_in = nn.Linear(in_size, hid_size)
        self.lin_out = nn.Linear(hid_size, out_size)
        self.linlayers = nn.ModuleList(nn.Linear(hid_size, hid_size)
                                       for _ in range(num_hid_layers))
        self.gcnlayers = nn.ModuleList(MaxKGCNConv(hid_size, hid_size, weight=False, maxk=maxk,
                                                   allow_zero_in_degree=True,
                                                   feat_drop=feat_drop)
                                       for _ in range(num_hid_layers))
        self.normlayers = nn.ModuleList(nn.LayerNorm(hid_size) for _ in range(num_hid_layers)
                                        ) if norm else None
        for lin in [self.lin_in, self.lin_out, *self.linlayers]:
            nn.init.xavier_uniform_(lin.weight)

    def forward(self, g, x):
        x = self.lin_in(x).relu()
        for i, conv in enumerate(self.gcnlayers):
            x = conv(g, self.linlayers[i](x))
            if self.normlayers is not None:
                x = self.normlayers[i](x)
        return self.lin_out(x)
