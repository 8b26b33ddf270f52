"""MaxKSAGEConv / MaxKGCNConv drop-ins.

CPU: CSRGraph construction (destination rows) and the GraphConv / SAGE edge weights.
GPU: each layer on the gfx950 kernels against a dense float64 torch restatement of the DGL
semantics the reference trained with (utils/models.py:12-26 MaxK, then dglnn.SAGEConv
'mean' / dglnn.GraphConv), forward and every gradient within 1e-5 norm-wise; a few optimiser steps
of MaxKSAGE / MaxKGCN reduce the loss. DGL is not installed here, so these dense
formulations stand in for it (parity with DGL itself is unpinned).
"""
import numpy as np
import pytest
import torch

import maxk_kernels as mk
from maxk_kernels import graphs
from maxk_kernels.layers import MaxKGCN, MaxKGCNConv, MaxKSAGE, MaxKSAGEConv


def small_edges(n=300, e=4000, seed=5):
    ptr, idx = graphs.synthetic_csr(n, e, seed=seed)
    rows = torch.repeat_interleave(torch.arange(n), (ptr[1:] - ptr[:-1]).long())
    return rows, idx.long(), n   # dst, src


# ------------------------------------------------------------------------ CPU
def test_from_edges_groups_by_destination():
    src = torch.tensor([0, 2, 1, 2, 3, 0])
    dst = torch.tensor([1, 1, 0, 3, 3, 3])
    g = mk.CSRGraph.from_edges(src, dst, 4)
    assert g.ptr.tolist() == [0, 1, 3, 3, 6]
    assert g.idx.tolist() == [1, 0, 2, 0, 2, 3]
    assert g.in_degrees().tolist() == [1, 2, 0, 3]
    assert g.out_degrees().tolist() == [2, 1, 2, 1]


def test_edge_values_match_dgl_norms():
    src = torch.tensor([0, 2, 1, 2, 3, 0])
    dst = torch.tensor([1, 1, 0, 3, 3, 3])
    g = mk.CSRGraph.from_edges(src, dst, 4)
    ind = g.in_degrees().clamp(min=1).double()
    outd = g.out_degrees().clamp(min=1).double()
    rows = torch.repeat_interleave(torch.arange(4), g.in_degrees())
    cols = g.idx.long()
    exp = {"sum": torch.ones(6, dtype=torch.float64), "mean": 1 / ind[rows],
           "right": 1 / ind[rows], "left": 1 / outd[cols],
           "both": outd[cols] ** -0.5 * ind[rows] ** -0.5}
    for kind, ref in exp.items():
        assert torch.allclose(g.edge_values(kind).double(), ref, rtol=1e-6), kind
    assert g.edge_values("both") is g.edge_values("both")          # cached
    assert g.with_values("mean").ptr is g.ptr                       # plan shared
    with pytest.raises(ValueError):
        g.edge_values("max")


# ------------------------------------------------------------------------ GPU helpers
def dense_adj(csr: mk.CSRGraph, kind: str) -> torch.Tensor:
    n = csr.num_nodes
    v = csr.edge_values(kind).double().cpu()
    return torch.sparse_csr_tensor(csr.ptr.long().cpu(), csr.idx.long().cpu(), v,
                                   size=(n, n)).to_dense()


def maxk_dense(x: torch.Tensor, k: int) -> torch.Tensor:
    """utils/models.py:12-26 (topk mask; differentiable)."""
    idx = torch.topk(x.detach(), k, dim=1).indices
    return x * torch.zeros_like(x).scatter_(1, idx, 1.0)


def close(a, b, tol=1e-5):
    """Norm-wise: max|a - b| <= tol * max|b|. The layers add f32 GEMMs (rocBLAS) around the
    aggregation, whose rounding on cancelling dot products is not an aggregation error;
    the element-wise 1e-5 bar on the kernels themselves is in test_gpu_parity.py."""
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max()) <= tol * float(b.abs().max())


@pytest.mark.gpu
@pytest.mark.parametrize("k", [8, 16, 32])
@pytest.mark.parametrize("agg", ["mean", "sum"])
def test_sage_conv_matches_dense(gpu, k, agg):
    dst, src, n = small_edges()
    csr = mk.CSRGraph.from_edges(src.to(gpu), dst.to(gpu), n)
    torch.manual_seed(0)
    conv = MaxKSAGEConv(64, 48, agg, maxk=k).to(gpu)
    with torch.no_grad():
        conv.bias.uniform_(-0.5, 0.5)
    x = graphs.features(n, 64, seed=3).to(gpu).requires_grad_(True)
    y = conv(csr, x)
    w = graphs.features(n, 48, seed=4).to(gpu)
    (y * w).sum().backward()

    xr = x.detach().cpu().double().requires_grad_(True)
    ws = conv.fc_self.weight.detach().cpu().double().requires_grad_(True)
    wn = conv.fc_neigh.weight.detach().cpu().double().requires_grad_(True)
    b = conv.bias.detach().cpu().double().requires_grad_(True)
    xm = maxk_dense(xr, k)
    yr = xm @ ws.T + (dense_adj(csr, agg) @ xm) @ wn.T + b      # dglnn.SAGEConv(mean|sum)
    (yr * w.cpu().double()).sum().backward()
    assert close(y, yr)
    assert close(x.grad, xr.grad)
    assert close(conv.fc_self.weight.grad, ws.grad)
    assert close(conv.fc_neigh.weight.grad, wn.grad)
    assert close(conv.bias.grad, b.grad)


@pytest.mark.gpu
def test_sage_conv_reference_ordering(gpu):
    """maxk_after_fc=True: the reference layer's h_self + A MaxK(fc_neigh(x))."""
    dst, src, n = small_edges()
    csr = mk.CSRGraph.from_edges(src.to(gpu), dst.to(gpu), n)
    torch.manual_seed(1)
    conv = MaxKSAGEConv(64, 64, "mean", maxk=16, bias=False, maxk_after_fc=True).to(gpu)
    x = graphs.features(n, 64, seed=3).to(gpu)
    y = conv(csr, x)
    xr = x.cpu().double()
    ws = conv.fc_self.weight.detach().cpu().double()
    wn = conv.fc_neigh.weight.detach().cpu().double()
    yr = xr @ ws.T + dense_adj(csr, "mean") @ maxk_dense(xr @ wn.T, 16)
    assert close(y, yr)


@pytest.mark.gpu
@pytest.mark.parametrize("norm", ["both", "right", "left", "none"])
def test_gcn_conv_matches_dense(gpu, norm):
    dst, src, n = small_edges(seed=7)
    csr = mk.CSRGraph.from_edges(src.to(gpu), dst.to(gpu), n)
    torch.manual_seed(2)
    conv = MaxKGCNConv(64, 32, norm=norm, maxk=16).to(gpu)
    with torch.no_grad():
        conv.bias.uniform_(-0.5, 0.5)
    x = graphs.features(n, 64, seed=6).to(gpu).requires_grad_(True)
    y = conv(csr, x)
    w = graphs.features(n, 32, seed=8).to(gpu)
    (y * w).sum().backward()

    xr = x.detach().cpu().double().requires_grad_(True)
    wt = conv.weight.detach().cpu().double().requires_grad_(True)
    b = conv.bias.detach().cpu().double().requires_grad_(True)
    yr = dense_adj(csr, norm) @ maxk_dense(xr @ wt, 16) + b     # dglnn.GraphConv(norm)
    (yr * w.cpu().double()).sum().backward()
    assert close(y, yr)
    assert close(x.grad, xr.grad)
    assert close(conv.weight.grad, wt.grad)
    assert close(conv.bias.grad, b.grad)


@pytest.mark.gpu
def test_gcn_conv_zero_in_degree_check(gpu):
    src = torch.tensor([0, 1], device=gpu)
    dst = torch.tensor([1, 0], device=gpu)
    csr = mk.CSRGraph.from_edges(src, dst, 3)       # node 2 has no in-edges
    conv = MaxKGCNConv(16, 16, maxk=4).to(gpu)
    with pytest.raises(ValueError, match="zero in-degree"):
        conv(csr, torch.randn(3, 16, device=gpu))
    conv.allow_zero_in_degree = True
    y = conv(csr, torch.randn(3, 16, device=gpu))
    assert torch.allclose(y[2], conv.bias)


@pytest.mark.gpu
@pytest.mark.parametrize("model_cls", [MaxKSAGE, MaxKGCN])
def test_model_trains(gpu, model_cls):
    dst, src, n = small_edges(n=800, e=16000, seed=11)
    csr = mk.CSRGraph.from_edges(src.to(gpu), dst.to(gpu), n)
    torch.manual_seed(3)
    feats = graphs.features(n, 32, seed=12).to(gpu)
    labels = torch.randint(0, 5, (n,), generator=torch.Generator().manual_seed(1)).to(gpu)
    model = model_cls(32, 64, 2, 5, maxk=16, feat_drop=0.1, norm=True).to(gpu)
    opt = torch.optim.Adam(model.parameters(), lr=0.01)
    losses = []
    for _ in range(30):
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(model(csr, feats), labels)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert np.isfinite(losses).all()
    assert losses[-1] < losses[0] - 0.1      # random labels: fitting, not generalising
