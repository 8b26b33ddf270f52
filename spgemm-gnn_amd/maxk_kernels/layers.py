"""Drop-in MaxK graph layers on the gfx950 SpGEMM / SSpMM kernels.

Replaces the reference's ``MaxKSAGEConv`` (utils/maxk_layers.py:47-265) and
``MaxKGCNConv`` (utils/maxk_layers.py:267-448) with the same constructor signatures, and
``MaxKSAGE`` / ``MaxKGCN`` / ``MaxKGIN`` (utils/integrated_models.py:8-271, imported by
maxk_gnn_integrated.py:21 and built with the kwargs of :317-332) with the same
constructors, but with the SURVEY §8(b) caller defects fixed:

* MaxK yields CBSR ``(sp_data, sp_index)`` directly; no dense ``[N, k]`` misuse, no
  per-row Python ``_extract_sparse_format`` loop, no uint8 wrap (D <= 256 is checked);
* the aggregation runs over the in-edge CSR (destination rows) and is differentiable:
  SpGEMM forward, SSpMM backward, MaxK backward scatter;
* edge weights are built on the device once per graph (no per-row ``.item()`` loop).

Numerics follow DGL on the same inputs (the semantics the reference trained with,
utils/models.py:109-411 + dglnn.SAGEConv / GraphConv / GINConv):

* ``nonlinear="maxk"`` (default): MaxK feeds the SpGEMM kernels.
  - ``MaxKSAGEConv``: ``rst = fc_self(x) + fc_neigh(mean_{u->v} x_u) (+ bias)``, then
    ``norm``; ``x = feat_drop(MaxK(feat))``. Dropout acts on the k kept values only (the
    other entries are zero either way). The reference's layer applies MaxK after
    ``fc_neigh`` and dropout to its output (maxk_layers.py:85-88,183);
    ``maxk_after_fc=True`` keeps that ordering.
  - ``MaxKGCNConv``: ``rst = A_norm MaxK(feat W) (+ bias)`` with ``A_norm`` the GraphConv
    normalisation ('both', 'right', 'left', 'none'); with ``weight=False`` this is
    ``dglnn.GraphConv(weight=None)`` applied to ``MaxK(feat)``.
  - ``MaxKGINConv``: ``rst = (1 + eps) x + sum_{u->v} x_u`` on ``x = MaxK(feat)``
    (``dglnn.GINConv(learn_eps=True, activation=None)``, utils/models.py:373).
* ``nonlinear="relu"`` (``--nonlinear relu``, utils/config.py:47): the models apply ReLU
  themselves and the layers aggregate the dense features with the HIP CSR SpMM
  (``maxk_dense_spmm_csr``; backward on the transposed CSR), i.e. the plain DGL layers
  of utils/models.py (``dglnn.SAGEConv(mean)``, ``GraphConv(weight=None)``, ``GINConv``).

``norm`` of ``MaxKSAGEConv`` may be a module instance (DGL's convention) or a class that is
instantiated as ``norm(out_feats)`` (utils/maxk_layers.py:66-67).

``graph`` may be a :class:`~maxk_kernels.autograd.CSRGraph` or a DGL graph (converted
with ``adj_tensors('csc')`` when DGL is installed; it is not required).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .autograd import CSRGraph, dense_aggregate, densify, maxk, maxk_aggregate, spgemm

NONLINEAR = ("maxk", "relu")


def as_csr(graph) -> CSRGraph:
    if isinstance(graph, CSRGraph):
        return graph
    if hasattr(graph, "adj_tensors"):
        return CSRGraph.from_dgl(graph)
    raise TypeError("graph must be a maxk_kernels.CSRGraph or a DGL graph")


def _check_nonlinear(nonlinear: str) -> str:
    if nonlinear not in NONLINEAR:
        raise ValueError(f"nonlinear must be one of {NONLINEAR} (utils/config.py:47), "
                         f"got {nonlinear!r}")
    return nonlinear


def _sparse_dropout(sp_data: torch.Tensor, p: float, training: bool) -> torch.Tensor:
    return F.dropout(sp_data, p, training) if p > 0 else sp_data


def _make_norm(norm, out_feats):
    """DGL passes a module instance; the reference layer passes a class and calls
    ``norm(out_feats)`` (utils/maxk_layers.py:66-67). Accept both."""
    if norm is None:
        return None
    if isinstance(norm, type):
        return norm(out_feats)
    return norm


class MaxKSAGEConv(nn.Module):
    """GraphSAGE layer with MaxK sparsity and the fused aggregation kernels.

    Signature of utils/maxk_layers.py:51-52 plus ``bias`` (dglnn.SAGEConv has one),
    ``maxk_after_fc`` (the reference layer's MaxK placement) and ``nonlinear``.
    """

    def __init__(self, in_feats, out_feats, aggregator_type="mean", feat_drop=0., norm=None,
                 maxk=32, bias=True, maxk_after_fc=False, topk_mode="exact",
                 nonlinear="maxk"):
        super().__init__()
        if aggregator_type not in ("mean", "sum"):
            raise ValueError(f"Unsupported aggregator type: {aggregator_type}")
        self.in_feats = in_feats
        self.out_feats = out_feats
        self.aggregator_type = aggregator_type
        self.maxk = maxk
        self.maxk_after_fc = maxk_after_fc
        self.topk_mode = topk_mode
        self.nonlinear = _check_nonlinear(nonlinear)
        self.fc_self = nn.Linear(in_feats, out_feats, bias=False)
        self.fc_neigh = nn.Linear(in_feats, out_feats, bias=False)
        self.bias = nn.Parameter(torch.zeros(out_feats)) if bias else None
        self.norm = _make_norm(norm, out_feats)
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
        if self.nonlinear == "relu":
            # dglnn.SAGEConv(mean) on dense features (the model applied the ReLU)
            x = F.dropout(feat, self.feat_drop, self.training) if self.feat_drop > 0 else feat
            rst = self.fc_self(x) + self.fc_neigh(dense_aggregate(x, csr))
        elif self.maxk_after_fc:
            # reference ordering (maxk_layers.py:85-88): MaxK(fc_neigh(feat)) aggregated
            h_self = self.fc_self(feat)
            if self.feat_drop > 0 and self.training:
                sp_data, sp_index = maxk(self.fc_neigh(feat), self.maxk, self.topk_mode)
                sp_data = _sparse_dropout(sp_data, self.feat_drop, self.training)
                rst = h_self + spgemm(sp_data, sp_index, csr, self.out_feats)
            else:  # no dropout between MaxK and the SpGEMM: the fused producer-consumer pair
                rst = h_self + maxk_aggregate(self.fc_neigh(feat), csr, self.maxk, self.topk_mode)
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
    ``feat_drop``: dropout between MaxK and the aggregation, as utils/models.py:262-264,
    and ``nonlinear``)."""

    def __init__(self, in_feats, out_feats, norm="both", weight=True, bias=True,
                 allow_zero_in_degree=False, maxk=32, topk_mode="exact", feat_drop=0.,
                 nonlinear="maxk"):
        super().__init__()
        if norm not in ("both", "right", "left", "none"):
            raise ValueError(f"Invalid norm value {norm!r}")
        self.in_feats = in_feats
        self.out_feats = out_feats
        self.norm = norm
        self.maxk = maxk
        self.topk_mode = topk_mode
        self.nonlinear = _check_nonlinear(nonlinear)
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
        if self.nonlinear == "relu":
            x = F.dropout(feat, self.feat_drop, self.training) if self.feat_drop > 0 else feat
            rst = dense_aggregate(x, csr.with_values(self.norm))
        elif self.feat_drop > 0 and self.training:
            sp_data, sp_index = maxk(feat, self.maxk, self.topk_mode)
            sp_data = _sparse_dropout(sp_data, self.feat_drop, self.training)
            rst = spgemm(sp_data, sp_index, csr.with_values(self.norm), feat.shape[1])
        else:
            rst = maxk_aggregate(feat, csr.with_values(self.norm), self.maxk, self.topk_mode)
        if self.bias is not None:
            rst = rst + self.bias
        return rst


class MaxKGINConv(nn.Module):
    """GIN layer (``dglnn.GINConv(learn_eps=True, activation=None)``, sum aggregator, no
    apply_func; utils/models.py:373) on MaxK features:
    ``rst = (1 + eps) x + sum_{u->v} x_u`` with ``x = feat_drop(MaxK(feat))`` through the
    SpGEMM kernels, or ``x = feat`` and the dense SpMM for ``nonlinear='relu'``."""

    def __init__(self, in_feats, out_feats=None, learn_eps=True, maxk=32, init_eps=0.,
                 topk_mode="exact", feat_drop=0., nonlinear="maxk"):
        super().__init__()
        if out_feats is not None and out_feats != in_feats:
            raise ValueError("GINConv without apply_func keeps the feature size")
        self.in_feats = in_feats
        self.maxk = maxk
        self.topk_mode = topk_mode
        self.feat_drop = float(feat_drop)
        self.nonlinear = _check_nonlinear(nonlinear)
        eps = torch.tensor([float(init_eps)])
        if learn_eps:
            self.eps = nn.Parameter(eps)
        else:
            self.register_buffer("eps", eps)

    def forward(self, graph, feat: torch.Tensor) -> torch.Tensor:
        csr = as_csr(graph).with_values("sum")
        if self.nonlinear == "relu":
            x = F.dropout(feat, self.feat_drop, self.training) if self.feat_drop > 0 else feat
            return (1 + self.eps) * x + dense_aggregate(x, csr)
        sp_data, sp_index = maxk(feat, self.maxk, self.topk_mode)
        sp_data = _sparse_dropout(sp_data, self.feat_drop, self.training)
        x = densify(sp_data, sp_index, self.in_feats)
        return (1 + self.eps) * x + spgemm(sp_data, sp_index, csr, self.in_feats)


class MaxKSAGE(nn.Module):
    """utils/integrated_models.py:8-66 (MaxK applied inside each MaxKSAGEConv); with
    ``nonlinear='relu'`` the utils/models.py:109-165 SAGE: ReLU, then dglnn.SAGEConv(mean)."""

    def __init__(self, in_size, hid_size, num_hid_layers, out_size, maxk=32, feat_drop=0.5,
                 norm=False, nonlinear="maxk"):
        super().__init__()
        self.nonlinear = _check_nonlinear(nonlinear)
        self.num_layers = num_hid_layers
        self.lin_in = nn.Linear(in_size, hid_size)
        self.lin_out = nn.Linear(hid_size, out_size)
        self.layers = nn.ModuleList(
            MaxKSAGEConv(hid_size, hid_size, "mean", feat_drop=feat_drop,
                         norm=nn.LayerNorm(hid_size) if norm else None, maxk=maxk,
                         nonlinear=nonlinear)
            for _ in range(num_hid_layers))
        nn.init.xavier_uniform_(self.lin_in.weight)
        nn.init.xavier_uniform_(self.lin_out.weight)

    def forward(self, g, x):
        x = self.lin_in(x)
        for layer in self.layers:
            if self.nonlinear == "relu":
                x = F.relu(x)
            x = layer(g, x)
        return self.lin_out(x)


class MaxKGCN(nn.Module):
    """utils/models.py:240-289 GCN (lin -> MaxK or ReLU -> dropout -> GraphConv(weight=None)
    -> LayerNorm)."""

    def __init__(self, in_size, hid_size, num_hid_layers, out_size, maxk=32, feat_drop=0.5,
                 norm=False, nonlinear="maxk"):
        super().__init__()
        self.nonlinear = _check_nonlinear(nonlinear)
        self.num_layers = num_hid_layers
        self.lin_in = nn.Linear(in_size, hid_size)
        self.lin_out = nn.Linear(hid_size, out_size)
        self.linlayers = nn.ModuleList(nn.Linear(hid_size, hid_size)
                                       for _ in range(num_hid_layers))
        self.gcnlayers = nn.ModuleList(MaxKGCNConv(hid_size, hid_size, weight=False, maxk=maxk,
                                                   allow_zero_in_degree=True,
                                                   feat_drop=feat_drop, nonlinear=nonlinear)
                                       for _ in range(num_hid_layers))
        self.normlayers = nn.ModuleList(nn.LayerNorm(hid_size) for _ in range(num_hid_layers)
                                        ) if norm else None
        for lin in [self.lin_in, self.lin_out, *self.linlayers]:
            nn.init.xavier_uniform_(lin.weight)

    def forward(self, g, x):
        x = self.lin_in(x).relu()
        for i, conv in enumerate(self.gcnlayers):
            x = self.linlayers[i](x)
            if self.nonlinear == "relu":
                x = F.relu(x)
            x = conv(g, x)
            if self.normlayers is not None:
                x = self.normlayers[i](x)
        return self.lin_out(x)


class MaxKGIN(nn.Module):
    """utils/models.py:363-411 GIN (lin -> MaxK or ReLU -> dropout -> GINConv(learn_eps)
    -> LayerNorm), the constructor of utils/integrated_models.py:145-149."""

    def __init__(self, in_size, hid_size, num_hid_layers, out_size, maxk=32, feat_drop=0.5,
                 norm=False, nonlinear="maxk"):
        super().__init__()
        self.nonlinear = _check_nonlinear(nonlinear)
        self.num_layers = num_hid_layers
        self.lin_in = nn.Linear(in_size, hid_size)
        self.lin_out = nn.Linear(hid_size, out_size)
        self.linlayers = nn.ModuleList(nn.Linear(hid_size, hid_size)
                                       for _ in range(num_hid_layers))
        self.ginlayers = nn.ModuleList(MaxKGINConv(hid_size, maxk=maxk, feat_drop=feat_drop,
                                                   nonlinear=nonlinear)
                                       for _ in range(num_hid_layers))
        self.normlayers = nn.ModuleList(nn.LayerNorm(hid_size) for _ in range(num_hid_layers)
                                        ) if norm else None
        for lin in [self.lin_in, self.lin_out, *self.linlayers]:
            nn.init.xavier_uniform_(lin.weight)

    def forward(self, g, x):
        x = self.lin_in(x).relu()
        for i, conv in enumerate(self.ginlayers):
            x = self.linlayers[i](x)
            if self.nonlinear == "relu":
                x = F.relu(x)
            x = conv(g, x)
            if self.normlayers is not None:
                x = self.normlayers[i](x)
        return self.lin_out(x)
