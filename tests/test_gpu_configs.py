"""GPU, the two BASELINE.json configs that have no kernel of their own in the bench:

* config 1 — "flickr GraphSAGE hidden=64 ReLU baseline on DGL CPU SpMM path": the ReLU
  layers' dense aggregation (maxk_kernels.dense_aggregate: HIP CSR SpMM forward, the same
  kernel on the transposed CSR backward) on the Flickr-shaped graph (N=89,250,
  E=989,006 + self-loops, synthetic), hidden 64, checked against the oracle's DGL
  update_all(copy_u, mean) restatement, plus a MaxKSAGE(nonlinear='relu') training step;
* config 5 — "Reddit row-partitioned across 8 x MI355X": the full-size RowPartition with
  every rank's rectangular plans run on this one GPU and the all-gather / reduce-scatter
  emulated with tensor ops (the real collectives are covered by tests/test_dist.py over
  gloo and test_gpu_dist.py over RCCL), for W in {2, 4, 8} and k in {16, 64}: every row of
  the forward and every column of the backward against the oracle, plus the adjoint identity.
"""
import time

import numpy as np
import pytest
import torch

import maxk_kernels as mk
from maxk_kernels import graphs
from maxk_kernels.dist import RowPartition
from oracle import oracle

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


def _transpose(ptr, idx, val):
    n = ptr.size - 1
    rows = np.repeat(np.arange(n, dtype=np.int32), np.diff(ptr))
    order = np.argsort(idx, kind="stable")
    pt = np.zeros(n + 1, np.int32)
    pt[1:] = np.cumsum(np.bincount(idx, minlength=n))
    return pt, rows[order], val[order]


def test_config1_flickr_relu_dense_aggregation(gpu):
    n, e = graphs.DATASETS["flickr"]
    ptr, idx = graphs.synthetic_csr(n, e, seed=97)
    p, ix = ptr.numpy(), idx.numpy()
    csr = mk.CSRGraph(ptr.to(gpu), idx.to(gpu)).with_values("mean")
    x = torch.relu(graphs.features(n, 64, seed=97))          # ReLU input, hidden 64
    g = graphs.features(n, 64, seed=98)
    xg = x.to(gpu).requires_grad_(True)
    y = mk.dense_aggregate(xg, csr)
    y.backward(g.to(gpu))
    torch.cuda.synchronize()
    # DGL update_all(copy_u, mean) (oracle, f32) and the per-element sum of |terms|
    ref = oracle.dense_spmm(p, ix, None, x.numpy(), mean=True)
    w = csr.val.cpu().numpy()
    mag = oracle.dense_spmm(p, ix, w, np.abs(x.numpy()))
    ok, worst = oracle.close_enough(y.detach().cpu().numpy(), ref, mag)
    assert ok, worst
    pt, it, wt = _transpose(p, ix, w)
    ref_b = oracle.dense_spmm(pt, it, wt, g.numpy())
    mag_b = oracle.dense_spmm(pt, it, wt, np.abs(g.numpy()))
    ok, worst = oracle.close_enough(xg.grad.cpu().numpy(), ref_b, mag_b)
    assert ok, worst
    # timing of the config-1 aggregation on the GPU (printed; the CPU figure is bench.py's
    # cpu_baseline / tools/cpu_config1.py)
    xd = x.to(gpu)
    for _ in range(3):
        mk.dense_aggregate(xd, csr)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        mk.dense_aggregate(xd, csr)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 20 * 1e3
    print(f"flickr hidden 64 dense aggregation (mean): {ms:.3f} ms, {e / ms / 1e6:.2f} G edges/s")


def test_config1_flickr_relu_sage_trains(gpu):
    """MaxKSAGE(nonlinear='relu') built as maxk_gnn_integrated.py:317-321 builds it, on the
    Flickr-shaped graph with Flickr's 500 input features and 7 classes: a few steps run and
    fit the (random) labels."""
    n, e = graphs.DATASETS["flickr"]
    ptr, idx = graphs.synthetic_csr(n, e, seed=97, device=gpu)
    csr = mk.CSRGraph(ptr, idx)
    torch.manual_seed(0)
    feats = graphs.features(n, 500, seed=3, device=gpu)
    labels = torch.randint(0, 7, (n,), device=gpu)
    model = mk.MaxKSAGE(500, 64, 3, 7, 32, feat_drop=0.2, norm=True, nonlinear="relu").to(gpu)
    opt = torch.optim.Adam(model.parameters(), lr=0.01)
    losses = []
    for _ in range(15):
        opt.zero_grad()
        loss = torch.nn.functional.cross_entropy(model(csr, feats), labels)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert np.isfinite(losses).all() and losses[-1] < losses[0]


_ORACLE5 = {}


def _config5_oracle(ptr, sp_data, sp_index, g, k, D):
    """The whole-graph oracle outputs (f64 sums and |terms| sums) for config 5 at this k,
    computed once and shared by the world sizes."""
    if _ORACLE5.get("k") != k:
        _ORACLE5.clear()
        idx = graphs.synthetic_rows(ptr, seed=97)
        val = graphs.sage_mean_values(ptr, num_edges=idx.numel())
        p, ix, v = ptr.cpu().numpy(), idx.cpu().numpy(), val.cpu().numpy()
        del idx, val
        si = sp_index.cpu().numpy()
        fwd = oracle.spgemm_forward(p, ix, v, sp_data.cpu().numpy(), si, D, with_mag=True)
        bwd = oracle.sspmm_backward(p, ix, v, g.cpu().numpy(), si, with_mag=True)
        _ORACLE5.update(k=k, fwd=fwd, bwd=bwd)
    return _ORACLE5["fwd"], _ORACLE5["bwd"]


def _close_in_chunks(got, ref, mag, rows=1 << 17):
    worst = 0.0
    for a in range(0, ref.shape[0], rows):
        ok, w = oracle.close_enough(got[a:a + rows], ref[a:a + rows], mag[a:a + rows])
        worst = max(worst, w)
        assert ok, (a, w)
    return worst


@pytest.mark.parametrize("k", [16, 64])
@pytest.mark.parametrize("W", [2, 4, 8])
def test_config5_reddit_partition(gpu, W, k):
    """BASELINE config 5 emulated on one GPU, the path the 8-GPU bench times: the bench graph
    (each rank generates only its rows), every rank's ShardedAggregation over the all-gathered
    record table (filled here as the one RCCL all-gather would, statistics pairs included), the
    reduce-scatter as a sum. EVERY row of the forward and EVERY column of the backward against
    the oracle's whole-graph f64 sums (oracle.close_enough: 1e-5 relative, 1e-5 of the |terms|
    sum where terms cancel), the worst error/bound printed per (W, k)."""
    from maxk_kernels.dist import ShardedAggregation, record_bytes, record_views
    D = 256
    n, e = graphs.DATASETS["reddit"]
    ptr = graphs.synthetic_ptr(n, e, seed=97, device=gpu)
    h = graphs.features(n, D, seed=97, device=gpu)
    g = graphs.features(n, D, seed=98, device=gpu)
    sp_data, sp_index = mk.maxk_forward(h, k, return_index=True)
    del h
    part = RowPartition(ptr, W)
    assert part.padded_rows >= n
    # the padded record table every rank holds after the forward exchange
    table_rec = torch.zeros((part.padded_rows, record_bytes(k)), dtype=torch.uint8, device=gpu)
    td, ti = record_views(table_rec, k)
    for q in range(W):
        a, b = part.rows(q)
        pos = part.table_positions(q, gpu)
        td[pos] = sp_data[a:b]
        ti[pos] = sp_index[a:b]
        mk.cbsr_stats(sp_data[a:b], sp_index[a:b],
                      out=table_rec.view(torch.int32)[part.stats_position(q), :2])
    y = torch.empty((n, D), device=gpu)
    grad_table = torch.zeros((part.padded_rows, k), device=gpu)
    ranks_e = []
    for q in range(W):
        a, b = part.rows(q)
        idx_q = graphs.synthetic_rows(ptr, seed=97, rows=(a, b))
        val_q = graphs.sage_mean_values(ptr[a:b + 1], num_edges=idx_q.numel())
        ranks_e.append(idx_q.numel())
        shard = ShardedAggregation(part, q, ptr, idx_q, val_q, D, k, local_edges=True)
        shard.table_rec.copy_(table_rec)
        y[a:b] = shard.compute_forward()
        grad_table += shard.compute_backward(g[a:b])                    # the reduce-scatter
        del shard
    torch.cuda.synchronize()
    gs = torch.cat([grad_table[part.table_positions(q, gpu)] for q in range(W)])
    del grad_table, table_rec
    # nnz balance of the partition: every rank within 1 % of E / W
    assert max(ranks_e) <= 1.01 * e / W and sum(ranks_e) == e
    # adjoint identity <A densify(sp), G> = <sp, SSpMM(G)>
    lhs = (y.double() * g.double()).sum().item()
    rhs = (sp_data.double() * gs.double()).sum().item()
    scale = (y.double().abs() * g.double().abs()).sum().item()
    assert abs(lhs - rhs) <= 1e-5 * scale
    (ref, mag), (gref, gmag) = _config5_oracle(ptr, sp_data, sp_index, g, k, D)
    wf = _close_in_chunks(y.cpu().numpy(), ref, mag)
    wb = _close_in_chunks(gs.cpu().numpy(), gref, gmag)
    print(f"config 5 reddit W={W} k={k}: forward every row worst err/bound {wf:.3g}; "
          f"backward every column worst err/bound {wb:.3g}")
    mk.clear_plan_cache()
