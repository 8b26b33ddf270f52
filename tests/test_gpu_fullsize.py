"""GPU, BASELINE full size (Reddit-shaped synthetic graph, D=256, k=16): parity through
size-independent properties plus sampled rows/columns checked against the oracle.

* adjoint identity   <A densify(sp), G> == <sp_data, SSpMM(G)>   (float64 reductions)
* linearity          SpGEMM(2 sp_data) == 2 SpGEMM(sp_data)
* sampled rows       forward rows vs the oracle on the induced sub-CSR
* sampled columns    backward columns vs the oracle on the columns' in-edges
"""
import numpy as np
import pytest
import torch

import maxk_kernels as mk
from maxk_kernels import graphs
from oracle import oracle

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

N, E = graphs.DATASETS["reddit"]
D, K = 256, 16


@pytest.fixture(scope="module")
def reddit(gpu):
    ptr, idx = graphs.synthetic_csr(N, E, seed=97, device=gpu)
    val = graphs.sage_mean_values(ptr)
    h = graphs.features(N, D, seed=97, device=gpu)
    g = graphs.features(N, D, seed=98, device=gpu)
    sp_data, sp_index = mk.maxk_forward(h, K, return_index=True)
    return ptr, idx, val, sp_data, sp_index, g


def test_graph_shape(reddit):
    ptr, idx = reddit[0], reddit[1]
    assert ptr.numel() == N + 1 and idx.numel() == E and int(ptr[-1]) == E


def test_adjoint_and_linearity(reddit):
    ptr, idx, val, sp_data, sp_index, g = reddit
    y, _ = mk.spgemm_forward(ptr, idx, val, sp_data, sp_index, N, E, K, D)
    gs = mk.spgemm_backward(ptr, idx, val, g, sp_index, N, E, K, D)
    lhs = (y.double() * g.double()).sum().item()
    rhs = (sp_data.double() * gs.double()).sum().item()
    scale = (y.double().abs() * g.double().abs()).sum().item()
    assert abs(lhs - rhs) <= 1e-5 * scale
    y2, _ = mk.spgemm_forward(ptr, idx, val, sp_data * 2, sp_index, N, E, K, D)
    mag = (y.abs() * 2).double()
    assert ((y2.double() - 2 * y.double()).abs() <= 1e-5 * mag + 1e-30).all()


def test_sampled_rows_vs_oracle(reddit):
    ptr, idx, val, sp_data, sp_index, _ = reddit
    y, _ = mk.spgemm_forward(ptr, idx, val, sp_data, sp_index, N, E, K, D)
    p = ptr.cpu().numpy()
    deg = np.diff(p)
    rows = np.unique(np.concatenate([np.random.RandomState(0).choice(N, 1500, replace=False),
                                     np.argsort(deg)[-8:]]))   # include the heaviest rows
    ix, v = idx.cpu().numpy(), val.cpu().numpy()
    sub_ptr = np.zeros(rows.size + 1, np.int64)
    sub_ptr[1:] = np.cumsum(deg[rows])
    sub_idx = np.concatenate([ix[p[r]:p[r + 1]] for r in rows])
    sub_val = np.concatenate([v[p[r]:p[r + 1]] for r in rows])
    # the oracle reads sp rows by column id: hand it the full CBSR table
    big_ptr = np.zeros(N + 1, np.int32)
    big_ptr[1:rows.size + 1] = sub_ptr[1:]
    big_ptr[rows.size + 1:] = sub_ptr[-1]
    ref, mag = oracle.spgemm_forward(big_ptr, sub_idx, sub_val, sp_data.cpu().numpy(),
                                     sp_index.cpu().numpy(), D, with_mag=True)
    ok, worst = oracle.close_enough(y[torch.from_numpy(rows).to(y.device)].cpu().numpy(),
                                    ref[:rows.size], mag[:rows.size])
    assert ok, worst


def test_sampled_columns_vs_oracle(reddit):
    ptr, idx, val, _, sp_index, g = reddit
    gs = mk.spgemm_backward(ptr, idx, val, g, sp_index, N, E, K, D)
    cols = np.random.RandomState(1).choice(N, 400, replace=False)
    ix = idx.cpu().numpy()
    sel = np.isin(ix, cols)
    e_ids = np.nonzero(sel)[0]
    rows_of = np.repeat(np.arange(N), np.diff(ptr.cpu().numpy()))[e_ids]
    c = ix[e_ids]
    v = val.cpu().numpy()[e_ids].astype(np.float64)
    si = sp_index.cpu().numpy()
    gn = g.cpu().numpy()
    ref = np.zeros((N, K))
    mag = np.zeros((N, K))
    terms = v[:, None] * gn[rows_of[:, None], si[c].astype(np.int64)]
    np.add.at(ref, c, terms)
    np.add.at(mag, c, np.abs(terms))
    ok, worst = oracle.close_enough(gs.cpu().numpy()[cols], ref[cols], mag[cols])
    assert ok, worst
