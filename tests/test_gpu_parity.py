"""GPU parity: the gfx950 kernels (through the C ABI) against the CPU oracle.

Bars (BASELINE.json north_star): top-k index output bit-exact (and its values, which are
copies); fp32 accumulators within 1e-5 relative: plain |got - ref| <= 1e-5 |ref| on every
element that does not cancel (|ref| >= half the sum of its |terms|), 1e-5 of that sum on
the ones that do (oracle.close_enough).
"""
import os

import numpy as np
import pytest
import torch

import maxk_kernels as mk
from maxk_kernels import graphs
from oracle import oracle

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "maxk_small.npz")
RTOL = 1e-5


@pytest.fixture(scope="module")
def golden():
    with np.load(GOLDEN, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def to_dev(a, dev, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.to(dev)


def assert_close(got, ref, mag, rtol=RTOL):
    got = got.detach().cpu().numpy() if torch.is_tensor(got) else got
    ok, worst = oracle.close_enough(got, ref, mag, rtol=rtol)
    rel = oracle.worst_relative(got, ref, mag)
    print(f"worst err/bound {worst:.3g}; worst |got-ref|/|ref| (non-cancelling) {rel:.3g}")
    assert ok, f"worst err/bound = {worst:.3g}, worst relative {rel:.3g}"


def graph_on(dev, ptr, idx, val):
    return to_dev(ptr, dev), to_dev(idx, dev), to_dev(val, dev)


def heavy_graph(n=6000, e=60_000, heavy_rows=(17, 4000), seed=21):
    """Synthetic graph plus rows connected to every node: rows longer than the forward
    task cap (4096) are split into segments (the atomic path)."""
    ptr, idx = graphs.synthetic_csr(n, e, seed=seed)
    rows = []
    p = ptr.numpy()
    ix = idx.numpy()
    for r in range(n):
        rows.append(np.arange(n, dtype=np.int32) if r in heavy_rows else ix[p[r]:p[r + 1]])
    deg = np.array([len(x) for x in rows])
    ptr2 = np.zeros(n + 1, np.int32)
    ptr2[1:] = np.cumsum(deg)
    idx2 = np.concatenate(rows).astype(np.int32)
    val = np.random.RandomState(seed).uniform(0.1, 1.0, idx2.size).astype(np.float32)
    return ptr2, idx2, val


def empty_rows_graph(n=3000, seed=22):
    rs = np.random.RandomState(seed)
    deg = rs.poisson(3, n)
    deg[rs.rand(n) < 0.3] = 0
    deg[:40] = 0        # a whole empty forward tile
    ptr = np.zeros(n + 1, np.int32)
    ptr[1:] = np.cumsum(deg)
    idx = np.concatenate([np.sort(rs.choice(n, d, replace=False)) for d in deg]).astype(np.int32)
    val = rs.randn(idx.size).astype(np.float32)
    return ptr, idx, val


# ------------------------------------------------------------------------ top-k
EDGE = os.path.join(os.path.dirname(__file__), "golden", "maxk_refcompat_edge.npz")


@pytest.mark.parametrize("k", [1, 8, 16, 32, 64])
def test_topk_ref_compat_edge_rows_bit_exact(gpu, k):
    """NaN / +-Inf / +-0 / all-equal / cap exits with cnt > k and cnt < k / denormals
    (tests/golden/make_golden.py:edge_rows), bit for bit including the sign of zero."""
    with np.load(EDGE, allow_pickle=False) as z:
        x, gd, gi = z["x"], z[f"data_k{k}"], z[f"index_k{k}"]
    d, i = mk.maxk_forward(to_dev(x, gpu), k, mode="ref_compat", return_index=True)
    assert np.array_equal(i.cpu().numpy(), gi)
    assert np.array_equal(d.cpu().numpy().view(np.uint32), gd.view(np.uint32))


NAN_ROWS = os.path.join(os.path.dirname(__file__), "golden", "maxk_exact_nan.npz")


@pytest.mark.parametrize("k", [1, 8, 16, 32, 64])
def test_topk_exact_nan_rows_bit_exact(gpu, k):
    """Exact mode on +-NaN rows (tests/golden/make_golden.py:nan_rows): every NaN ranks above
    +Inf, NaNs tie at the lowest index, as torch.topk (tests/test_oracle.py checks the fixture
    against it); bit for bit, NaN payloads included, in the plain and the record layouts."""
    with np.load(NAN_ROWS, allow_pickle=False) as z:
        x, gd, gi = z["x"], z[f"data_k{k}"], z[f"index_k{k}"]
    d, i = mk.maxk_forward(to_dev(x, gpu), k, mode="exact", return_index=True)
    assert np.array_equal(i.cpu().numpy(), gi)
    assert np.array_equal(d.cpu().numpy().view(np.uint32), gd.view(np.uint32))


@pytest.mark.parametrize("k", [8, 16, 24, 32, 64])
@pytest.mark.parametrize("mode", ["exact", "ref_compat"])
def test_topk_golden_bit_exact(gpu, golden, k, mode):
    h = to_dev(golden["h"], gpu)
    d, i = mk.maxk_forward(h, k, mode=mode, return_index=True)
    pre = "exact" if mode == "exact" else "ref"
    assert np.array_equal(i.cpu().numpy(), golden[f"{pre}_index_k{k}"])
    assert np.array_equal(d.cpu().numpy(), golden[f"{pre}_data_k{k}"])


@pytest.mark.parametrize("d", [256, 128, 64, 100, 7])
@pytest.mark.parametrize("mode", ["exact", "ref_compat"])
def test_topk_random_bit_exact(gpu, d, mode):
    x = graphs.features(4099, d, seed=d)
    x[5, :] = 0.5                                   # a fully tied row
    x[6, : d // 2] = -0.0
    for k in sorted({1, min(d, 3), min(d, 16), min(d, 32), d}):
        gd, gi = mk.maxk_forward(x.to(gpu), k, mode=mode, return_index=True)
        od, oi = oracle.maxk(x.numpy(), k, mode)
        assert np.array_equal(gi.cpu().numpy(), oi), (d, k)
        assert np.array_equal(gd.cpu().numpy(), od), (d, k)


@pytest.mark.parametrize("d,k", [(100, 5), (256, 64), (37, 37)])
def test_topk_eight_rows_per_wave_bit_exact(gpu, d, k):
    """N >= 2^20 rows takes the 8-rows-per-wave exact kernel (maxk_topk.hip kTopkRows8),
    including a ragged last wave, odd k (byte-stored selectors) and k == D."""
    n = (1 << 20) + 3
    x = graphs.features(n, d, seed=k)
    x[n - 1, :] = 0.25                              # tied row in the ragged last wave
    gd, gi = mk.maxk_forward(x.to(gpu), k, mode="exact", return_index=True)
    od, oi = oracle.maxk(x.numpy(), k, "exact")
    assert np.array_equal(gi.cpu().numpy(), oi)
    assert np.array_equal(gd.cpu().numpy(), od)


def _offset_view(t: torch.Tensor, gpu) -> torch.Tensor:
    """A contiguous copy of ``t`` whose storage starts one element past an allocation
    boundary (4-B misaligned floats/ints, odd byte address for u8)."""
    buf = torch.empty(t.numel() + 1, dtype=t.dtype, device=gpu)
    v = buf[1:].view(t.shape)
    v.copy_(t.to(gpu))
    assert v.is_contiguous() and v.data_ptr() % 16 != 0
    return v


@pytest.mark.parametrize("k", [8, 16, 32, 24])
def test_offset_views_through_every_entry_point(gpu, k):
    """Contiguous tensors need not be 16-B aligned (a view one element into a buffer): the
    top-k, both aggregation directions (plan built from offset graph tensors too) and the
    MaxK scatter give the aligned results."""
    p, ix, v = GRAPHS["synthetic"]()
    n, d = p.size - 1, 256
    x = graphs.features(n, d, seed=k)
    g = graphs.features(n, d, seed=k + 1)
    od, oi = oracle.maxk(x.numpy(), k)
    for mode in ("exact", "ref_compat"):
        md, mi = oracle.maxk(x.numpy(), k, mode)
        sd = _offset_view(torch.zeros(n, k), gpu)
        si = _offset_view(torch.zeros(n, k, dtype=torch.uint8), gpu)
        mk.maxk_forward(_offset_view(x, gpu), k, mode=mode, out=(sd, si))
        assert np.array_equal(si.cpu().numpy(), mi), mode
        assert np.array_equal(sd.cpu().numpy(), md), mode
    ptr, idx, val = (_offset_view(torch.from_numpy(a), gpu) for a in (p, ix, v))
    sd, si = _offset_view(torch.from_numpy(od), gpu), _offset_view(torch.from_numpy(oi), gpu)
    ref, mag = oracle.spgemm_forward(p, ix, v, od, oi, d, with_mag=True)
    out, _ = mk.spgemm_forward(ptr, idx, val, sd, si, n, ix.size, k, d)
    assert_close(out, ref, mag)
    ref, mag = oracle.sspmm_backward(p, ix, v, g.numpy(), oi, with_mag=True)
    gs = mk.spgemm_backward(ptr, idx, val, _offset_view(g, gpu), si, n, ix.size, k, d)
    assert_close(gs, ref, mag)
    gin = mk.maxk_backward(_offset_view(gs, gpu), si, dim_origin=d)
    assert np.array_equal(gin.cpu().numpy(), oracle.maxk_backward(gs.cpu().numpy(), oi, d))
    dense = oracle.maxk_backward(od, oi, d)  # densified CBSR rows
    ref = oracle.dense_spmm(p, ix, v, dense)
    mag = oracle.dense_spmm(p, ix, np.abs(v), np.abs(dense))
    y = mk.dense_spmm(ptr, idx, val, _offset_view(torch.from_numpy(dense), gpu))
    assert_close(y, ref, mag, rtol=2e-6 * 64)  # f32 sums in two orders (test_dense_spmm_vs_oracle)


@pytest.mark.parametrize("levels", [4, 16, 256])
@pytest.mark.parametrize("k", [8, 16, 32, 64])
def test_topk_ties_vs_torch_topk(gpu, levels, k):
    """Tie-heavy rows (features quantised to a few levels): the exact mode's selection against
    torch.topk on the same device, the top-k the reference trained with (utils/models.py:14,
    ``x.topk(k, dim=1)``). Both must select the same multiset of values; where a tie at the
    k-th value lets them pick different indices, ours is the lowest-index choice (the oracle's
    rule, bit-exact), and the share of such rows is reported."""
    n, d = 20_000, 256
    x = graphs.features(n, d, seed=levels + k)
    x = torch.round(x * (levels / 8.0)) / (levels / 8.0)     # ~levels distinct values per row
    xg = x.to(gpu)
    sd, si = mk.maxk_forward(xg, k, mode="exact", return_index=True)
    tv, ti = torch.topk(xg, k, dim=1)
    # same selected values (as a multiset) per row
    assert torch.equal(torch.sort(sd, dim=1).values, torch.sort(tv, dim=1).values)
    ours = torch.zeros_like(xg, dtype=torch.bool).scatter_(1, si.long(), True)
    theirs = torch.zeros_like(xg, dtype=torch.bool).scatter_(1, ti, True)
    differ = (ours != theirs).any(dim=1)
    # ours: bit-exact with the lowest-index rule
    od, oi = oracle.maxk(x.numpy(), k)
    assert np.array_equal(si.cpu().numpy(), oi)
    # where the sets differ, the k-th value is tied across the boundary
    kth = tv[:, -1:]
    on_tie = ((ours ^ theirs) & ~(xg == kth)).any(dim=1)
    assert not on_tie.any()
    print(f"ties: levels={levels} k={k}: torch.topk picked other indices on "
          f"{int(differ.sum())} of {n} rows ({100.0 * differ.float().mean().item():.2f} %)")


def test_topk_default_returns_reference_shape(gpu):
    x = graphs.features(10, 64, seed=1).to(gpu)
    out = mk.maxk_forward(x, 16)
    assert out.shape == (10, 16) and out.dtype == torch.float32


@pytest.mark.parametrize("k", [8, 16, 24, 32, 64])
def test_maxk_backward_golden(gpu, golden, k):
    gs = to_dev(golden[f"bwd_k{k}"], gpu)
    i = to_dev(golden[f"exact_index_k{k}"], gpu)
    out = mk.maxk_backward(gs, i, dim_origin=256)
    assert np.array_equal(out.cpu().numpy(), golden[f"maxk_bwd_k{k}"])


def test_maxk_backward_repeated_index_and_reference_width(gpu):
    g = torch.tensor([[1.0, 2.0, 3.0], [4.0, 5.0, 6.0]], device=gpu)
    i = torch.tensor([[4, 1, 4], [0, 2, 9]], device=gpu, dtype=torch.int64)
    out = mk.maxk_backward(g, i)          # reference width: max(indices) + 1 = 10
    assert out.shape == (2, 10)
    ref = oracle.maxk_backward(g.cpu().numpy(), i.cpu().numpy().astype(np.uint8), 10)
    assert np.array_equal(out.cpu().numpy(), ref)


# ------------------------------------------------------------------------ SpGEMM forward
@pytest.mark.parametrize("k", [16, 24])
def test_spgemm_forward_golden(gpu, golden, k):
    ptr, idx, val = graph_on(gpu, golden["ptr"], golden["idx"], golden["val"])
    d = to_dev(golden[f"exact_data_k{k}"], gpu)
    i = to_dev(golden[f"exact_index_k{k}"], gpu)
    n = ptr.numel() - 1
    out, si = mk.spgemm_forward(ptr, idx, val, d, i, n, idx.numel(), k, 256)
    assert si is i
    assert_close(out, golden[f"fwd_k{k}"], golden[f"fwd_mag_k{k}"])


GRAPHS = {
    "synthetic": lambda: (lambda p, i: (p.numpy(), i.numpy(),
                                        graphs.sage_mean_values(p).numpy()))(
        *graphs.synthetic_csr(5000, 120_000, seed=31)),
    "heavy_split": heavy_graph,
    # community structure in ID order (column locality): GCN values
    "community": lambda: (lambda p, i: (p.numpy(), i.numpy(),
                                        graphs.gcn_values(p, i).numpy()))(
        *graphs.community_csr(6000, 150_000, communities=12, seed=33)),
    "empty_rows": empty_rows_graph,
    "single_node": lambda: (np.array([0, 1], np.int32), np.array([0], np.int32),
                            np.array([0.5], np.float32)),
    # no edges at all: the forward must still write zeros, the backward zeros
    "no_edges": lambda: (np.zeros(70, np.int32), np.zeros(0, np.int32), np.zeros(0, np.float32)),
}


@pytest.mark.parametrize("gname", list(GRAPHS))
@pytest.mark.parametrize("d,k", [(256, 8), (256, 16), (256, 32), (256, 64), (256, 24),
                                 (64, 16), (100, 10), (128, 70), (256, 256)])
def test_spgemm_forward_vs_oracle(gpu, gname, d, k):
    p, ix, v = GRAPHS[gname]()
    n = p.size - 1
    x = graphs.features(n, d, seed=k)
    od, oi = oracle.maxk(x.numpy(), k)
    ref, mag = oracle.spgemm_forward(p, ix, v, od, oi, d, with_mag=True)
    ptr, idx, val = graph_on(gpu, p, ix, v)
    out, _ = mk.spgemm_forward(ptr, idx, val, to_dev(od, gpu), to_dev(oi, gpu), n, ix.size,
                               k, d)
    assert_close(out, ref, mag)


@pytest.mark.parametrize("n,row", [(48, 47), (48, 32), (33, 32), (64, 63), (100, 70), (48, 39),
                                   (80, 78)])
@pytest.mark.parametrize("d,k", [(1, 1), (256, 16), (256, 8), (256, 32)])
def test_spgemm_forward_edgeless_tiles_before_edges(gpu, n, row, d, k):
    """Every row before `row` is edgeless, so whole forward tiles share their (empty) first
    edge with the tile that owns the edges; the edges must still land in `row` (found by
    tests/test_gpu_fuzz.py: a tile ordered after its edgeless neighbour lost its edges)."""
    rs = np.random.RandomState(n + row)
    p = np.zeros(n + 1, np.int32)
    p[row + 1:] = min(n, 40)
    ix = np.sort(rs.choice(n, min(n, 40), replace=False)).astype(np.int32)
    v = rs.randn(ix.size).astype(np.float32)
    x = graphs.features(n, d, seed=k)
    od, oi = oracle.maxk(x.numpy(), k)
    ref, mag = oracle.spgemm_forward(p, ix, v, od, oi, d, with_mag=True)
    ptr, idx, val = graph_on(gpu, p, ix, v)
    out, _ = mk.spgemm_forward(ptr, idx, val, to_dev(od, gpu), to_dev(oi, gpu), n, ix.size, k, d)
    assert_close(out, ref, mag)


def test_spgemm_forward_duplicate_selectors_summed(gpu):
    p = np.array([0, 2, 3], np.int32)
    ix = np.array([0, 1, 1], np.int32)
    v = np.array([1.0, 2.0, 0.5], np.float32)
    data = np.array([[1.0, 10.0, 2.0, 3.0], [3.0, 4.0, 1.0, 1.0]], np.float32)
    index = np.array([[5, 5, 5, 1], [0, 7, 7, 7]], np.uint8)
    ref, mag = oracle.spgemm_forward(p, ix, v, data, index, 8, with_mag=True)
    ptr, idx, val = graph_on(gpu, p, ix, v)
    out, _ = mk.spgemm_forward(ptr, idx, val, to_dev(data, gpu), to_dev(index, gpu), 2, 3, 4, 8)
    assert_close(out, ref, mag)
    for fixed in (1, 2):   # pair chunks: both selectors of a chunk name the same slot
        plan = mk.GraphPlan(ptr, idx, val, 2, 3, 8, 4,
                            options={"fwd_chunk3": 3, "fwd_fixed": fixed})
        assert_close(plan.forward(to_dev(data, gpu), to_dev(index, gpu)), ref, mag)


@pytest.mark.parametrize("gname", ["synthetic", "heavy_split", "empty_rows", "single_node",
                                   "no_edges"])
@pytest.mark.parametrize("k", [2, 6, 8, 10, 14, 16, 18, 24, 32, 64, 128])
@pytest.mark.parametrize("mode", ["exact", "ref_compat"])
def test_spgemm_forward_pair_chunks_vs_oracle(gpu, gname, k, mode):
    """Pair-chunk records (the k = 16 default, fwd_chunk3 = 3 at any even k up
    to 128): quad-shared edge words when k / 2 % 4 == 0, the pack fused into the statistics
    pass when k % 4 == 0 and on its own otherwise; fixed point and f64 accumulation; ref_compat
    tables (rows with fewer than k entries over the threshold repeat selector 0 with value 0)."""
    p, ix, v = GRAPHS[gname]()
    n, d = p.size - 1, 256
    x = graphs.features(n, d, seed=k + 11)
    if mode == "ref_compat":
        x[::3, : d // 2] = 0.0   # few entries above the bisection threshold on these rows
    od, oi = oracle.maxk(x.numpy(), k, mode=mode)
    ref, mag = oracle.spgemm_forward(p, ix, v, od, oi, d, with_mag=True)
    ptr, idx, val = graph_on(gpu, p, ix, v)
    for fixed in (0, 1, 2):
        plan = mk.GraphPlan(ptr, idx, val, n, ix.size, d, k,
                            options={"fwd_chunk3": 3, "fwd_fixed": fixed})
        assert plan.info()["fwd_layout"] == 4
        assert_close(plan.forward(to_dev(od, gpu), to_dev(oi, gpu)), ref, mag)


def _fwd_both_paths(gpu, p, ix, v, od, oi, d, k, **opts):
    n = p.size - 1
    ptr, idx, val = graph_on(gpu, p, ix, v)
    outs = []
    for fixed in (1, 2):
        plan = mk.GraphPlan(ptr, idx, val, n, ix.size, d, k, options=dict(opts, fwd_fixed=fixed))
        outs.append(plan.forward(to_dev(od, gpu), to_dev(oi, gpu)).cpu().numpy())
    return outs


@pytest.mark.parametrize("gname", ["synthetic", "community", "empty_rows"])
@pytest.mark.parametrize("k", [8, 16, 32, 64])
def test_spgemm_forward_fixed_point_vs_f64_path(gpu, gname, k):
    """The fixed-point accumulation (fwd_fixed, the default) against the oracle, at the
    north_star bar and at the bound it guarantees (2^-24 of the f32 result on terms that do
    not cancel, plus the final f32 rounding); it must really run (its rounding differs from
    the f64 path's in some last bits)."""
    p, ix, v = GRAPHS[gname]()
    d = 256
    x = graphs.features(p.size - 1, d, seed=k + 5)
    od, oi = oracle.maxk(x.numpy(), k)
    ref, mag = oracle.spgemm_forward(p, ix, v, od, oi, d, with_mag=True)
    fixed, f64 = _fwd_both_paths(gpu, p, ix, v, od, oi, d, k)
    assert_close(fixed, ref, mag)
    assert_close(f64, ref, mag)
    assert oracle.worst_relative(fixed, ref, mag) <= 2.0 ** -24 + 2.0 ** -23
    if ix.size > 10_000:
        assert not np.array_equal(fixed, f64)


def test_spgemm_forward_fixed_point_bitwise_reproducible(gpu):
    """Integer sums do not depend on the order of the LDS atomics, and the bounds come from
    fixed-order row sums: every call of every plan of a graph gives the same bits."""
    p, ix, v = GRAPHS["heavy_split"]()
    n, d, k = p.size - 1, 256, 32
    od, oi = oracle.maxk(graphs.features(n, d, seed=12).numpy(), k)
    ptr, idx, val = graph_on(gpu, p, ix, v)
    sd, si = to_dev(od, gpu), to_dev(oi, gpu)
    outs = []
    for _ in range(2):
        plan = mk.GraphPlan(ptr, idx, val, n, ix.size, d, k, options={"fwd_fixed": 1})
        for _ in range(2):
            outs.append(plan.forward(sd, si).cpu().numpy().view(np.uint32))
    for o in outs[1:]:
        assert np.array_equal(o, outs[0])


@pytest.mark.parametrize("scale", [2.0 ** 24, 2.0 ** -24])
def test_spgemm_forward_fixed_point_follows_value_refresh(gpu, scale):
    """The per-task fixed-point bounds are plan state: refresh_values must recompute them (a
    stale 2^49 budget with values 2^24 times larger would overflow the integer sums; 2^24
    times smaller would lose 24 bits)."""
    p, ix, v = GRAPHS["synthetic"]()
    n, d, k = p.size - 1, 256, 16
    od, oi = oracle.maxk(graphs.features(n, d, seed=9).numpy(), k)
    ptr, idx, val = graph_on(gpu, p, ix, v)
    plan = mk.GraphPlan(ptr, idx, val, n, ix.size, d, k, options={"fwd_fixed": 1})
    v2 = (v * np.float32(scale)).astype(np.float32)
    plan.refresh_values(to_dev(v2, gpu))
    out = plan.forward(to_dev(od, gpu), to_dev(oi, gpu))
    ref, mag = oracle.spgemm_forward(p, ix, v2, od, oi, d, with_mag=True)
    assert_close(out, ref, mag)
    assert oracle.worst_relative(out.cpu().numpy(), ref, mag) <= 2.0 ** -24 + 2.0 ** -23


@pytest.mark.parametrize("case", ["wide_range", "inf", "nan", "zeros"])
def test_spgemm_forward_fixed_point_falls_back(gpu, case):
    """Inputs the fixed-point bound cannot cover take the f64 path: bitwise the same output
    as fwd_fixed=2 (a dynamic range of 2^40 in |x|; non-finite values; all zeros)."""
    p, ix, v = GRAPHS["synthetic"]()
    n, d, k = p.size - 1, 256, 16
    x = graphs.features(n, d, seed=3)
    od, oi = oracle.maxk(x.numpy(), k)
    od = od.copy()
    if case == "wide_range":
        od[::7] *= np.float32(2.0 ** -40)
    elif case == "inf":
        od[11, 3] = np.inf
    elif case == "nan":
        od[12, 0] = np.nan
    else:
        od[:] = 0.0
    fixed, f64 = _fwd_both_paths(gpu, p, ix, v, od, oi, d, k)
    assert np.array_equal(fixed.view(np.uint32), f64.view(np.uint32))
    if case == "wide_range":
        ref, mag = oracle.spgemm_forward(p, ix, v, od, oi, d, with_mag=True)
        assert_close(fixed, ref, mag)


# ------------------------------------------------------------------------ SSpMM backward
@pytest.mark.parametrize("k", [8, 16, 24, 32, 64])
def test_sspmm_backward_golden(gpu, golden, k):
    ptr, idx, val = graph_on(gpu, golden["ptr"], golden["idx"], golden["val"])
    g = to_dev(golden["g"], gpu)
    i = to_dev(golden[f"exact_index_k{k}"], gpu)
    n = ptr.numel() - 1
    gs = mk.spgemm_backward(ptr, idx, val, g, i, n, idx.numel(), k, 256)
    assert gs.shape == (n, k)
    assert_close(gs, golden[f"bwd_k{k}"], golden[f"bwd_mag_k{k}"])


@pytest.mark.parametrize("gname", list(GRAPHS))
@pytest.mark.parametrize("d,k", [(256, 8), (256, 16), (256, 32), (256, 64), (256, 24),
                                 (64, 16), (100, 10), (128, 70), (256, 256), (256, 5), (256, 250)])
def test_sspmm_backward_vs_oracle(gpu, gname, d, k):
    p, ix, v = GRAPHS[gname]()
    n = p.size - 1
    x = graphs.features(n, d, seed=k)
    g = graphs.features(n, d, seed=k + 1)
    _, oi = oracle.maxk(x.numpy(), k)
    ref, mag = oracle.sspmm_backward(p, ix, v, g.numpy(), oi, with_mag=True)
    ptr, idx, val = graph_on(gpu, p, ix, v)
    gs = mk.spgemm_backward(ptr, idx, val, g.to(gpu), to_dev(oi, gpu), n, ix.size, k, d)
    assert_close(gs, ref, mag)


@pytest.mark.parametrize("gname", list(GRAPHS))
@pytest.mark.parametrize("k", [4, 8, 24, 16])
def test_sspmm_backward_two_slots_vs_oracle(gpu, gname, k):
    """Two selector slots per lane (k/2 lanes per edge): the k=8 default on graphs whose
    column blocks see few edges per row (Reddit), forced here on every test graph; k=4 and
    k=24 take the non-quad record loads (2 and 12 lanes per edge)."""
    p, ix, v = GRAPHS[gname]()
    n, d = p.size - 1, 256
    x = graphs.features(n, d, seed=k)
    g = graphs.features(n, d, seed=k + 1)
    _, oi = oracle.maxk(x.numpy(), k)
    ref, mag = oracle.sspmm_backward(p, ix, v, g.numpy(), oi, with_mag=True)
    ptr, idx, val = graph_on(gpu, p, ix, v)
    plan = mk.GraphPlan(ptr, idx, val, n, ix.size, d, k, options=dict(bwd_features_per_lane=2))
    assert_close(plan.backward(g.to(gpu), to_dev(oi, gpu)), ref, mag)


@pytest.mark.parametrize("gname", list(GRAPHS))
@pytest.mark.parametrize("d,k", [(256, 1), (256, 3), (256, 7), (256, 13), (64, 17), (256, 61),
                                 (256, 130), (256, 199), (256, 255)])
@pytest.mark.parametrize("feats", [0, 4, 2])
def test_sspmm_backward_padded_slots_vs_oracle(gpu, gname, d, k, feats):
    """k that is not a multiple of the slots per lane F: the column-block kernel pads the
    selector slots to a multiple of F (padding slots gather feature 0 into accumulators
    that are never stored), with the default F, four and two slots per lane; every element of
    grad_sp is written, and value refreshes reach the records."""
    p, ix, v = GRAPHS[gname]()
    n = p.size - 1
    x = graphs.features(n, d, seed=k)
    g = graphs.features(n, d, seed=k + 1)
    _, oi = oracle.maxk(x.numpy(), k)
    ref, mag = oracle.sspmm_backward(p, ix, v, g.numpy(), oi, with_mag=True)
    ptr, idx, val = graph_on(gpu, p, ix, v)
    opts = dict(bwd_algo=1) if feats == 0 else dict(bwd_algo=1, bwd_features_per_lane=feats)
    plan = mk.GraphPlan(ptr, idx, val, n, ix.size, d, k, options=opts)
    gs = torch.full((n, k), float("nan"), device=gpu)
    plan.backward(g.to(gpu), to_dev(oi, gpu), gs)
    assert_close(gs, ref, mag)
    val.mul_(-2.0)                        # refresh_values rewrites the records' values
    ref, mag = oracle.sspmm_backward(p, ix, v * -2.0, g.numpy(), oi, with_mag=True)
    plan.refresh_values(val)
    assert_close(plan.backward(g.to(gpu), to_dev(oi, gpu)), ref, mag)


@pytest.mark.parametrize("gname", list(GRAPHS))
@pytest.mark.parametrize("d,k", [(256, 4), (256, 8), (256, 16), (256, 32), (256, 64), (256, 128),
                                 (256, 24), (100, 8), (64, 16), (256, 256)])
def test_sspmm_backward_twopass_vs_oracle(gpu, gname, d, k):
    """Two-pass backward (bwd_algo=3: row pass into the E x k workspace, column pass); k=24
    (6 lanes per edge) and edgeless graphs fall back to the blocks."""
    p, ix, v = GRAPHS[gname]()
    n = p.size - 1
    x = graphs.features(n, d, seed=k)
    g = graphs.features(n, d, seed=k + 1)
    _, oi = oracle.maxk(x.numpy(), k)
    ref, mag = oracle.sspmm_backward(p, ix, v, g.numpy(), oi, with_mag=True)
    ptr, idx, val = graph_on(gpu, p, ix, v)
    plan = mk.GraphPlan(ptr, idx, val, n, ix.size, d, k, options=dict(bwd_algo=3))
    assert plan.info()["bwd_algo"] == (1 if k == 24 or ix.size == 0 else 3)
    assert_close(plan.backward(g.to(gpu), to_dev(oi, gpu)), ref, mag)
    val.mul_(-2.0)                        # refresh_values rewrites the CSR-order records
    ref, mag = oracle.sspmm_backward(p, ix, v * -2.0, g.numpy(), oi, with_mag=True)
    plan.refresh_values(val)
    assert_close(plan.backward(g.to(gpu), to_dev(oi, gpu)), ref, mag)


def test_sspmm_backward_auto_twopass_on_sparse_wide_graph(gpu):
    """A graph whose column blocks would see each grad_out row about once (2 edges per row,
    60k columns) gets the two-pass backward by default; the forced block kernel agrees."""
    n, e, k, d = 60_000, 120_000, 16, 256
    ptr, idx = graphs.synthetic_csr(n, e, seed=41)
    p, ix = ptr.numpy(), idx.numpy()
    v = np.random.RandomState(41).uniform(-1.0, 1.0, ix.size).astype(np.float32)
    x = graphs.features(n, d, seed=42)
    g = graphs.features(n, d, seed=43)
    _, oi = oracle.maxk(x.numpy(), k)
    ref, mag = oracle.sspmm_backward(p, ix, v, g.numpy(), oi, with_mag=True)
    dptr, didx, dval = graph_on(gpu, p, ix, v)
    plan = mk.GraphPlan(dptr, didx, dval, n, ix.size, d, k)
    assert plan.info()["bwd_algo"] == 3
    assert_close(plan.backward(g.to(gpu), to_dev(oi, gpu)), ref, mag)
    forced = mk.GraphPlan(dptr, didx, dval, n, ix.size, d, k, options=dict(bwd_algo=1))
    assert forced.info()["bwd_algo"] == 1
    assert_close(forced.backward(g.to(gpu), to_dev(oi, gpu)), ref, mag)


@pytest.mark.parametrize("algo", [0, 1, 3])
@pytest.mark.parametrize("k", [16, 32])
def test_unsorted_rows_and_multi_edges(gpu, algo, k):
    """CSR rows with shuffled column order and repeated (row, column) edges: every edge
    counts once per occurrence in both directions, whatever the backward kernel."""
    rs = np.random.RandomState(55)
    p, ix, v = GRAPHS["synthetic"]()
    ix = ix.copy()
    for r in range(p.size - 1):                       # shuffle each row's columns
        rs.shuffle(ix[p[r]:p[r + 1]])
    rows = np.repeat(np.arange(p.size - 1), np.diff(p))
    dup = rs.rand(ix.size) < 0.1                      # repeat ~10 % of the edges in their row
    rows = np.concatenate([rows, rows[dup]])
    cols = np.concatenate([ix, ix[dup]])
    vals = np.concatenate([v, rs.uniform(-1, 1, dup.sum()).astype(np.float32)])
    order = np.argsort(rows, kind="stable")
    rows, cols, vals = rows[order], cols[order].astype(np.int32), vals[order]
    n, d = p.size - 1, 256
    p2 = np.zeros(n + 1, np.int32)
    p2[1:] = np.cumsum(np.bincount(rows, minlength=n))
    x = graphs.features(n, d, seed=56)
    g = graphs.features(n, d, seed=57)
    od, oi = oracle.maxk(x.numpy(), k)
    ref_f, mag_f = oracle.spgemm_forward(p2, cols, vals, od, oi, d, with_mag=True)
    ref_b, mag_b = oracle.sspmm_backward(p2, cols, vals, g.numpy(), oi, with_mag=True)
    ptr, idx, val = graph_on(gpu, p2, cols, vals)
    plan = mk.GraphPlan(ptr, idx, val, n, cols.size, d, k, options=dict(bwd_algo=algo))
    assert_close(plan.forward(to_dev(od, gpu), to_dev(oi, gpu)), ref_f, mag_f)
    assert_close(plan.backward(g.to(gpu), to_dev(oi, gpu)), ref_b, mag_b)


def test_plan_picks_up_value_changes(gpu):
    p, ix, v = GRAPHS["synthetic"]()
    n = p.size - 1
    ptr, idx, val = graph_on(gpu, p, ix, v)
    x = graphs.features(n, 256, seed=3)
    g = graphs.features(n, 256, seed=4)
    od, oi = oracle.maxk(x.numpy(), 16)
    d_sp, i_sp, gg = to_dev(od, gpu), to_dev(oi, gpu), g.to(gpu)
    mk.spgemm_backward(ptr, idx, val, gg, i_sp, n, ix.size, 16, 256)
    val.mul_(3.0)                         # in place: same pointer, new _version
    v3 = val.cpu().numpy()
    gs = mk.spgemm_backward(ptr, idx, val, gg, i_sp, n, ix.size, 16, 256)
    ref, mag = oracle.sspmm_backward(p, ix, v3, g.numpy(), oi, with_mag=True)
    assert_close(gs, ref, mag)
    out, _ = mk.spgemm_forward(ptr, idx, val, d_sp, i_sp, n, ix.size, 16, 256)
    ref, mag = oracle.spgemm_forward(p, ix, v3, od, oi, 256, with_mag=True)
    assert_close(out, ref, mag)


def test_plan_info(gpu):
    ptr, idx, val = graph_on(gpu, *heavy_graph())
    plan = mk.get_plan(ptr, idx, val, ptr.numel() - 1, idx.numel(), 256, 16)
    info = plan.info()
    assert info["fwd_split_rows"] == 2
    assert info["bwd_blocks"] * info["bwd_block_cols"] >= ptr.numel() - 1
    assert info["fwd_tasks"] > 0 and info["bwd_tasks"] >= info["bwd_blocks"]


@pytest.mark.parametrize("n,d,rows", [(120_000, 256, 39), (50_000, 256, 32), (120_000, 128, 32),
                                      (130_000, 212, 32), (130_000, 213, 47)])
def test_forward_tile_rows_default(gpu, n, d, rows):
    """Default forward tile: the most rows two work-groups per CU hold in LDS
    (39 at D = 256) where the 32-row tile already allowed only two (D >= 213) and the graph
    has rows for >= 5 rounds of them (>= 10 x 256 CUs x rows), else 32. Four edges per row, so
    fwd_tasks = ceil(n / rows); the 39- and 47-row forwards checked against the oracle."""
    rs = np.random.RandomState(n + d)
    p = (np.arange(n + 1, dtype=np.int64) * 4).astype(np.int32)
    ix = rs.randint(0, n, p[-1]).astype(np.int32)
    v = rs.rand(ix.size).astype(np.float32)
    ptr, idx, val = graph_on(gpu, p, ix, v)
    plan = mk.GraphPlan(ptr, idx, val, n, ix.size, d, 16)
    assert plan.info()["fwd_tasks"] == -(-n // rows)
    if rows > 32:
        x = graphs.features(n, d, seed=d)
        od, oi = oracle.maxk(x.numpy(), 16)
        ref, mag = oracle.spgemm_forward(p, ix, v, od, oi, d, with_mag=True)
        assert_close(plan.forward(to_dev(od, gpu), to_dev(oi, gpu)), ref, mag)


# ------------------------------------------------------------------------ autograd
def test_autograd_matches_dense_torch(gpu):
    p, ix, v = GRAPHS["synthetic"]()
    n = p.size - 1
    d, k = 64, 16
    x = graphs.features(n, d, seed=8).double()
    w = graphs.features(n, d, seed=9).double()
    graph = mk.CSRGraph(*graph_on(gpu, p, ix, v))
    xg = x.float().to(gpu).requires_grad_(True)
    y = mk.maxk_aggregate(xg, graph, k)
    loss = (y.double() * w.to(gpu)).sum()
    loss.backward()
    # dense float64 reference: topk mask -> A @ (x*mask)
    xr = x.clone().requires_grad_(True)
    idx_t = torch.topk(xr.detach(), k, dim=1).indices
    mask = torch.zeros_like(xr).scatter_(1, idx_t, 1.0)
    a = torch.sparse_csr_tensor(torch.from_numpy(p).long(), torch.from_numpy(ix).long(),
                                torch.from_numpy(v).double(), size=(n, n)).to_dense()
    yr = a @ (xr * mask)
    (yr * w).sum().backward()
    assert torch.allclose(y.double().cpu(), yr.detach(), rtol=1e-5, atol=1e-5)
    assert torch.allclose(xg.grad.double().cpu(), xr.grad, rtol=1e-5, atol=1e-5)


# ------------------------------------------------------------------------ dense comparator
def test_dense_spmm_vs_oracle(gpu):
    p, ix, v = GRAPHS["heavy_split"]()
    n = p.size - 1
    x = graphs.features(n, 64, seed=2)
    ref = oracle.dense_spmm(p, ix, v, x.numpy())          # f32 sums (DGL semantics)
    mag = oracle.dense_spmm(p, ix, np.abs(v), np.abs(x.numpy()))
    ptr, idx, val = graph_on(gpu, p, ix, v)
    y = mk.dense_spmm(ptr, idx, val, x.to(gpu))
    # both sides accumulate in f32 in different orders: bound by the summed magnitude
    assert_close(y, ref, mag, rtol=2e-6 * 64)


# ------------------------------------------------------------------------ plan options
# every maxk_plan_options knob the C ABI exposes selects a different kernel organisation;
# each must give the same results (the defaults are covered above)
PLAN_OPTIONS = [
    dict(fwd_tile_rows=16), dict(fwd_tile_rows=1), dict(fwd_tile_rows=64), dict(fwd_task_cap=512),
    dict(fwd_rotate=2), dict(fwd_rot_windows=64), dict(fwd_rot_windows=3, fwd_rot_rate=1),
    dict(bwd_unroll=12), dict(bwd_unroll=16), dict(bwd_waves=12), dict(bwd_waves=8, bwd_unroll=16), dict(bwd_waves=12, bwd_unroll=12),
    dict(bwd_waves=16), dict(bwd_waves=16, bwd_features_per_lane=2),
    dict(bwd_waves=16, bwd_piece_edges=500, bwd_slot_groups=2),
    # window hand-out: static interleave or an LDS counter, forward and backward
    dict(bwd_handout=1), dict(bwd_handout=2), dict(bwd_handout=2, bwd_piece_edges=500, bwd_waves=12),
    dict(bwd_handout=2, bwd_features_per_lane=2), dict(fwd_handout=2), dict(fwd_handout=2, fwd_rotate=2),
    dict(fwd_handout=2, fwd_tile_rows=1),
    # 8 waves per forward work-group, static and counter hand-out, one-row tiles
    dict(fwd_waves=8), dict(fwd_waves=8, fwd_handout=1), dict(fwd_waves=8, fwd_tile_rows=1),
    dict(fwd_waves=8, fwd_chunk3=1), dict(fwd_waves=8, fwd_fixed=2), dict(fwd_waves=4),
    dict(fwd_unroll=4), dict(fwd_waves=8, fwd_unroll=4, fwd_handout=1),
    dict(fwd_waves=8, fwd_unroll=4, fwd_chunk3=1),
    dict(bwd_slot_groups=2), dict(bwd_slot_groups=4), dict(bwd_lds_bytes=4096),
    dict(bwd_tasks_per_cu=1), dict(bwd_algo=3), dict(bwd_algo="two_pass"),
    # the accepted spellings of the defaults of removed knobs
    dict(fwd_accumulator="f64", bwd_accumulator="f32_cas", fwd_unroll=8, fwd_waves=4,
         bwd_acc_pad=2, bwd_sel_lds=1, fwd_prefetch=2, bwd_prefetch=2, fwd_branchless=1,
         bwd_cas64=1, bwd_tp_store=1, bwd_chunk_bounds=2, fwd_phases=1),
    # chunked blocks (slab flush by default, atomic flush into a memset grad_sp with
    # bwd_flush=1)
    dict(bwd_tasks_per_cu=32, bwd_min_task_edges=256),
    dict(bwd_tasks_per_cu=32, bwd_min_task_edges=256, bwd_flush=1),
    dict(bwd_tasks_per_cu=32, bwd_min_task_edges=256, bwd_flush=2, external_workspace=1),
    dict(bwd_tasks_per_cu=64, bwd_min_task_edges=16, bwd_features_per_lane=2),
    # pieces: every (block, chunk) task cut into pieces of <= 500 edges (slab regions per
    # piece), with chunks, slot groups, two slots per lane and the atomic flush
    dict(bwd_piece_edges=500), dict(bwd_piece_edges=500, bwd_tasks_per_cu=32, bwd_min_task_edges=256),
    dict(bwd_piece_edges=500, bwd_slot_groups=2), dict(bwd_piece_edges=500, bwd_features_per_lane=2),
    dict(bwd_piece_edges=500, bwd_flush=1),
    # XCD row windows of the task order, with chunks and pieces
    dict(bwd_order=2), dict(bwd_order=3), dict(bwd_order=2, bwd_tasks_per_cu=32, bwd_min_task_edges=256),
    dict(bwd_order=2, bwd_piece_edges=500, bwd_slot_groups=2),
    # two slots per lane (k/2 lanes per edge): unrolls, slot groups, chunks, more waves
    dict(bwd_features_per_lane=2), dict(bwd_features_per_lane=2, bwd_unroll=8),
    dict(bwd_features_per_lane=2, bwd_unroll=16), dict(bwd_features_per_lane=2, bwd_slot_groups=2),
    dict(bwd_features_per_lane=2, bwd_waves=12),
    dict(bwd_features_per_lane=2, bwd_tasks_per_cu=32, bwd_min_task_edges=256),
    dict(bwd_tasks_per_cu=32, bwd_min_task_edges=256, bwd_slot_groups=2),
    dict(bwd_waves=12, bwd_tasks_per_cu=32, bwd_min_task_edges=256),
    # lane-chunk forward records, two tables, fixed point / f64 with each forward layout
    dict(fwd_chunk3=1), dict(fwd_chunk3=2), dict(fwd_chunk3=1, fwd_fixed=2),
    # pair-chunk forward records {2 values, 2 selectors} (round 6), fixed point and f64, 4 / 8
    # waves (odd k falls back to the default layouts)
    dict(fwd_chunk3=3), dict(fwd_chunk3=3, fwd_fixed=2), dict(fwd_chunk3=3, fwd_waves=8),
    dict(fwd_chunk3=3, fwd_tile_rows=1), dict(fwd_tile_rows=39), dict(fwd_tile_rows=39, fwd_chunk3=3),
    dict(fwd_tile_rows=47, fwd_chunk3=2),
    dict(fwd_two_tables=1), dict(fwd_two_tables=2), dict(fwd_two_tables=1, fwd_fixed=2),
    dict(fwd_fixed=2), dict(fwd_fixed=1, fwd_chunk3=1), dict(fwd_fixed=1, fwd_tile_rows=64),
    dict(fwd_fixed=1, fwd_two_tables=1), dict(fwd_fixed=1, fwd_rotate=2),
    # column orders of the backward blocks (scattered, identity) with chunks, pieces, the
    # two-slot kernel, slot groups and the two-pass (which ignores them)
    dict(col_order="scattered"), dict(col_order="identity"),
    dict(col_order="scattered", bwd_tasks_per_cu=32, bwd_min_task_edges=256),
    dict(col_order="scattered", bwd_tasks_per_cu=32, bwd_min_task_edges=256, bwd_flush=1),
    dict(col_order="scattered", bwd_features_per_lane=2, bwd_tasks_per_cu=32, bwd_min_task_edges=256),
    dict(col_order="scattered", bwd_slot_groups=2, bwd_piece_edges=500),
    dict(col_order="scattered", bwd_lds_bytes=4096), dict(col_order="scattered", bwd_algo=3),
    # two-pass row chunks
    dict(bwd_algo=3, bwd_tp_chunks=2), dict(bwd_algo=3, bwd_tp_chunks=5),
    # row order inside the block streams (ascending / scattered) with chunks, pieces, slot
    # groups and a column order
    dict(bwd_row_order=1), dict(bwd_row_order=2, bwd_tasks_per_cu=32, bwd_min_task_edges=256),
    dict(bwd_row_order=2, col_order="scattered", bwd_slot_groups=2, bwd_piece_edges=500),
    dict(bwd_row_order=2, bwd_features_per_lane=2, bwd_tasks_per_cu=64, bwd_min_task_edges=16),
]

# option values refused with MAXK_ERR_UNSUPPORTED since ABI 3 (measured slower everywhere,
# never auto-selected) and values that were never valid
REMOVED_OPTIONS = [
    dict(fwd_accumulator="f32_cas"), dict(bwd_accumulator="f64"), dict(bwd_features_per_lane=1),
    dict(fwd_phases=3), dict(fwd_persistent=1), dict(fwd_unroll=16), dict(bwd_order=1),
    dict(bwd_acc_pad=1), dict(bwd_sel_lds=2), dict(bwd_algo=2),
    dict(fwd_prefetch=1), dict(bwd_prefetch=1), dict(fwd_record_bytes=256), dict(fwd_branchless=2),
    dict(bwd_cas64=2), dict(quad_loads=1), dict(quad_loads=2), dict(bwd_chunk_bounds=1),
    dict(bwd_chunk_bounds=3), dict(bwd_tp_store=2), dict(bwd_row_cost=8), dict(col_order=3),
]
INVALID_OPTIONS = [
    dict(bwd_unroll=7), dict(bwd_unroll=4), dict(bwd_slot_groups=3), dict(fwd_tile_rows=65),
    dict(bwd_lds_bytes=1 << 20), dict(bwd_algo=4), dict(bwd_waves=20), dict(fwd_chunk3=4),
    dict(bwd_handout=3), dict(fwd_handout=-1), dict(fwd_waves=6), dict(fwd_waves=16),
    dict(fwd_waves=4, fwd_unroll=4),
    dict(fwd_two_tables=3), dict(bwd_flush=3), dict(bwd_piece_edges=-1), dict(bwd_chunk_bounds=4),
    dict(col_order=5), dict(col_order=4), dict(bwd_tp_chunks=-2), dict(bwd_row_order=3),
    dict(bwd_features_per_lane=3), dict(fwd_fixed=3), dict(external_workspace=2), dict(bwd_order=4), dict(fwd_rotate=3),
]


@pytest.mark.parametrize("k,fw,fu,fh", [(8, 8, 8, 2), (16, 8, 8, 2), (32, 8, 8, 2), (48, 8, 4, 2),
                                         (64, 8, 8, 2)])
def test_plan_info_reports_launch_shapes(gpu, k, fw, fu, fh):
    """Defaults: 8 forward waves with the counter hand-out, 4
    sub-steps at k = 48; pair chunks at k = 16 (8 waves; the packed records that replace them
    with fwd_chunk3 = 2 take 4); 16 backward waves with the counter."""
    p, ix, v = GRAPHS["heavy_split"]()
    n = p.size - 1
    ptr, idx, val = graph_on(gpu, p, ix, v)
    info = mk.GraphPlan(ptr, idx, val, n, ix.size, 256, k).info()
    assert (info["fwd_waves"], info["fwd_unroll"], info["fwd_handout"]) == (fw, fu, fh)
    if k == 16:
        assert info["fwd_layout"] == 4
        rec = mk.GraphPlan(ptr, idx, val, n, ix.size, 256, k, options={"fwd_chunk3": 2}).info()
        assert rec["fwd_waves"] == 4 and rec["fwd_layout"] in (0, 1)  # tables: few edges/column
    assert (info["bwd_waves"], info["bwd_unroll"], info["bwd_handout"]) == (16, 8, 2)
    st = mk.GraphPlan(ptr, idx, val, n, ix.size, 256, k, options={"bwd_handout": 1}).info()
    assert st["bwd_waves"] in (8, 12) and st["bwd_handout"] == 1


@pytest.mark.parametrize("opts", PLAN_OPTIONS, ids=lambda o: ",".join(f"{k}={v}" for k, v in o.items()))
@pytest.mark.parametrize("k", [16, 32])
def test_plan_options_vs_oracle(gpu, opts, k):
    p, ix, v = GRAPHS["heavy_split"]()
    n, d = p.size - 1, 256
    x = graphs.features(n, d, seed=k)
    g = graphs.features(n, d, seed=k + 1)
    od, oi = oracle.maxk(x.numpy(), k)
    ref_f, mag_f = oracle.spgemm_forward(p, ix, v, od, oi, d, with_mag=True)
    ref_b, mag_b = oracle.sspmm_backward(p, ix, v, g.numpy(), oi, with_mag=True)
    ptr, idx, val = graph_on(gpu, p, ix, v)
    plan = mk.GraphPlan(ptr, idx, val, n, ix.size, d, k, options=opts)
    assert_close(plan.forward(to_dev(od, gpu), to_dev(oi, gpu)), ref_f, mag_f)
    assert_close(plan.backward(g.to(gpu), to_dev(oi, gpu)), ref_b, mag_b)


@pytest.mark.parametrize("fpl", [4, 2])
def test_slab_flush_reproducible(gpu, fpl):
    """Chunked column blocks with the slab flush: the combine adds the chunk partials in
    chunk order, so two calls agree bitwise (the atomic flush only to the oracle bar), and
    chunks that hold no edges still store their (zero) block."""
    p, ix, v = GRAPHS["heavy_split"]()
    n, d, k = p.size - 1, 256, 16
    g = graphs.features(n, d, seed=5)
    od, oi = oracle.maxk(graphs.features(n, d, seed=4).numpy(), k)
    ref_b, mag_b = oracle.sspmm_backward(p, ix, v, g.numpy(), oi, with_mag=True)
    ptr, idx, val = graph_on(gpu, p, ix, v)
    opts = dict(bwd_tasks_per_cu=64, bwd_min_task_edges=16, bwd_features_per_lane=fpl)
    plan = mk.GraphPlan(ptr, idx, val, n, ix.size, d, k, options=opts)
    info = plan.info()
    assert info["bwd_shared_blocks"] > 0
    gi = to_dev(oi, gpu)
    a = plan.backward(g.to(gpu), gi)
    b = torch.full_like(a, float("nan"))  # every element must be written
    plan.backward(g.to(gpu), gi, b)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    assert_close(a, ref_b, mag_b)


@pytest.mark.parametrize("bad", REMOVED_OPTIONS + INVALID_OPTIONS,
                         ids=lambda o: ",".join(f"{k}={v}" for k, v in o.items()))
def test_plan_options_rejected(gpu, bad):
    p, ix, v = GRAPHS["single_node"]()
    ptr, idx, val = graph_on(gpu, p, ix, v)
    with pytest.raises(RuntimeError) as exc:
        mk.GraphPlan(ptr, idx, val, 1, 1, 256, 16, options=bad)
    if bad in REMOVED_OPTIONS:
        assert "removed in ABI 3" in str(exc.value) and "code -2" in str(exc.value)


# ------------------------------------------------------------------------ rocSPARSE comparator
def test_rocsparse_comparator_vs_oracle(gpu):
    from maxk_kernels import baselines
    p, ix, v = GRAPHS["synthetic"]()
    n = p.size - 1
    x = graphs.features(n, 64, seed=4)
    ref = oracle.dense_spmm(p, ix, v, x.numpy())
    mag = oracle.dense_spmm(p, ix, np.abs(v), np.abs(x.numpy()))
    ptr, idx, val = graph_on(gpu, p, ix, v)
    y, ms = baselines.spmm_rocsparse(ptr, idx, val, x.to(gpu), times=2)
    assert ms > 0
    assert_close(y, ref, mag, rtol=2e-6 * 64)



@pytest.mark.parametrize("alg", ["default", "coo_segmented", "coo_atomic", "coo_segmented_atomic"])
def test_rocsparse_coo_comparator_vs_oracle(gpu, alg):
    from maxk_kernels import baselines
    p, ix, v = GRAPHS["synthetic"]()
    n = p.size - 1
    x = graphs.features(n, 64, seed=4)
    ref = oracle.dense_spmm(p, ix, v, x.numpy())
    mag = oracle.dense_spmm(p, ix, np.abs(v), np.abs(x.numpy()))
    ptr, idx, val = graph_on(gpu, p, ix, v)
    rows = baselines.coo_rows(ptr)
    assert rows.numel() == idx.numel()
    y, ms = baselines.spmm_rocsparse_coo(rows, idx, val, x.to(gpu), times=2, alg=alg)
    assert ms > 0
    assert_close(y, ref, mag, rtol=2e-6 * 64)


# ------------------------------------------------------------------------ streams / scratch
def test_two_streams_share_one_plan(gpu):
    """One cached plan used from two streams at once: each call takes its scratch (packed
    records, selector words) from the caching allocator on its own stream, so concurrent
    forward/backward calls on different inputs all match the oracle."""
    ptr, idx = graphs.synthetic_csr(20_000, 3_000_000, seed=31)
    val = graphs.sage_mean_values(ptr)
    n, d, k = 20_000, 256, 16
    dptr, didx, dval = ptr.to(gpu), idx.to(gpu), val.to(gpu)
    plan = mk.get_plan(dptr, didx, dval, n, idx.numel(), d, k)
    assert plan.fwd_ws_bytes > 0 and plan.bwd_ws_bytes > 0
    xs = [graphs.features(n, d, seed=40 + j) for j in range(2)]
    gs = [graphs.features(n, d, seed=50 + j) for j in range(2)]
    sps = [oracle.maxk(x.numpy(), k) for x in xs]
    streams = [torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)]
    torch.cuda.synchronize()
    outs = [[], []]
    for rep in range(3):
        for j, s in enumerate(streams):
            with torch.cuda.stream(s):
                sd, si = to_dev(sps[j][0], gpu), to_dev(sps[j][1], gpu)
                y, _ = mk.spgemm_forward(dptr, didx, dval, sd, si, n, idx.numel(), k, d)
                g = mk.spgemm_backward(dptr, didx, dval, to_dev(gs[j].numpy(), gpu), si, n,
                                       idx.numel(), k, d)
                outs[j].append((y, g))
    torch.cuda.synchronize()
    for j in range(2):
        ref, mag = oracle.spgemm_forward(ptr.numpy(), idx.numpy(), val.numpy(), *sps[j], d,
                                         with_mag=True)
        gref, gmag = oracle.sspmm_backward(ptr.numpy(), idx.numpy(), val.numpy(),
                                           gs[j].numpy(), sps[j][1], with_mag=True)
        for y, g in outs[j]:
            assert_close(y, ref, mag)
            assert_close(g, gref, gmag)


def test_value_refresh_is_ordered_after_other_streams(gpu):
    """In-place edge-value edits re-snapshot the cached plan on the editing stream only
    after the plan's earlier uses on other streams: a forward queued on stream A keeps the
    old values, the one on stream B after the edit sees the new ones."""
    ptr, idx = graphs.synthetic_csr(30_000, 3_000_000, seed=33)
    val = graphs.sage_mean_values(ptr)
    n, d, k = 30_000, 256, 16
    dptr, didx, dval = ptr.to(gpu), idx.to(gpu), val.to(gpu)
    od, oi = oracle.maxk(graphs.features(n, d, seed=60).numpy(), k)
    sd, si = to_dev(od, gpu), to_dev(oi, gpu)
    mk.spgemm_forward(dptr, didx, dval, sd, si, n, idx.numel(), k, d)   # build the plan
    torch.cuda.synchronize()
    a, b = torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)
    with torch.cuda.stream(a):
        ys = [mk.spgemm_forward(dptr, didx, dval, sd, si, n, idx.numel(), k, d)[0]
              for _ in range(6)]                                          # a long queue on A
    with torch.cuda.stream(b):
        dval.mul_(2.0)
        y2, _ = mk.spgemm_forward(dptr, didx, dval, sd, si, n, idx.numel(), k, d)
    torch.cuda.synchronize()
    ref, mag = oracle.spgemm_forward(ptr.numpy(), idx.numpy(), val.numpy(), od, oi, d,
                                     with_mag=True)
    for y in ys:
        assert_close(y, ref, mag)
    assert_close(y2, 2 * ref, 2 * mag)


def test_capi_external_workspace_contract(gpu):
    """A plan created with external_workspace holds no scratch: the plain entry points
    refuse it, the *_ws ones take a caller buffer of maxk_plan_workspace_bytes (and refuse
    a smaller one)."""
    import ctypes
    from maxk_kernels import _lib
    ptr, idx = graphs.synthetic_csr(5000, 200_000, seed=35)
    val = graphs.sage_mean_values(ptr)
    n, d, k = 5000, 256, 16
    dptr, didx, dval = ptr.to(gpu), idx.to(gpu), val.to(gpu)
    od, oi = oracle.maxk(graphs.features(n, d, seed=61).numpy(), k)
    sd, si = to_dev(od, gpu), to_dev(oi, gpu)
    plan = mk.GraphPlan(dptr, didx, dval, n, idx.numel(), d, k, options={"fwd_two_tables": 2})
    assert plan.fwd_ws_bytes >= n * 128            # one 128-B packed record per node (+ the
    #                                                fixed-point forward's 256-B stats slot)
    out = torch.empty((n, d), device=gpu)
    P = ctypes.c_void_p
    s = P(torch.cuda.current_stream().cuda_stream)
    args = (plan.handle, P(dptr.data_ptr()), P(didx.data_ptr()), P(dval.data_ptr()),
            P(sd.data_ptr()), P(si.data_ptr()), P(out.data_ptr()), n, idx.numel(), k, d)
    assert _lib.lib.maxk_spgemm_forward(*args, s) == -1
    small = torch.empty(plan.fwd_ws_bytes - 16, dtype=torch.uint8, device=gpu)
    assert _lib.lib.maxk_spgemm_forward_ws(*args, 0, P(small.data_ptr()), small.numel(), s) == -1
    ws = torch.empty(plan.fwd_ws_bytes, dtype=torch.uint8, device=gpu)
    assert _lib.lib.maxk_spgemm_forward_ws(*args, 0, P(ws.data_ptr()), ws.numel(), s) == 0
    torch.cuda.synchronize()
    ref, mag = oracle.spgemm_forward(ptr.numpy(), idx.numpy(), val.numpy(), od, oi, d,
                                     with_mag=True)
    assert_close(out, ref, mag)


def test_ref_compat_padding_slots_carry_no_gradient(gpu):
    """Rows where the reference bisection fills fewer than k slots: the (0.0f, 0) padding
    slots must not write a gradient into feature 0 unless feature 0 was selected."""
    k, d = 16, 256
    rs = np.random.RandomState(7)
    x = rs.rand(64, d).astype(np.float32)
    x[::2, 123] = 1e6          # even rows: one hit, 15 padding slots; feature 0 not selected
    x[1::4, 0] = 5e6           # rows 1, 5, ...: feature 0 is the single hit
    xt = to_dev(x, gpu).requires_grad_(True)
    sp_data, sp_index = mk.maxk(xt, k, mode="ref_compat")
    w = torch.randn(64, k, device=gpu)
    (sp_data * w).sum().backward()
    od, oi = oracle.maxk(x, k, "ref_compat")
    assert np.array_equal(sp_index.cpu().numpy(), oi)
    expect = np.zeros_like(x)
    wn = w.cpu().numpy()
    for r in range(64):
        for j in range(k):
            if od[r, j] != 0 or (j == 0 and x[r, oi[r, 0]] > 0):   # a filled slot
                expect[r, oi[r, j]] = wn[r, j]
    assert np.array_equal(xt.grad.cpu().numpy(), expect)


# ------------------------------------------------------------ fused top-k -> forward (round 6)
def _stat_rows(n, d, seed):
    """Random rows plus rows whose statistics are special: all zero, +-Inf, NaN of both signs,
    denormals, a single spike (ref_compat fills one slot and pads the rest)."""
    x = graphs.features(n, d, seed=seed)
    x[3] = 0.0
    x[4, 7] = float("inf")
    x[5, 9] = -float("inf")
    x[6, 11] = float("nan")
    x[7] = torch.from_numpy(np.array([0xffc00000] * d, np.uint32).view(np.float32))
    x[8] = 1e-40
    x[9, 100] = 1e6
    return x


@pytest.mark.parametrize("k", [1, 8, 16, 24, 32, 64])
@pytest.mark.parametrize("mode", ["exact", "ref_compat"])
@pytest.mark.parametrize("records", [False, True])
def test_topk_fused_stats_equal_cbsr_stats(gpu, k, mode, records):
    """maxk_topk_cbsr_ex (stats=): the pair fused into the top-k equals maxk_cbsr_stats over
    the emitted table bit for bit, and the table equals the plain top-k's, on random rows and
    rows with zeros, +-Inf, +-NaN, denormals and ref_compat padding (the special rows one at a
    time, so each sets the pair), in the plain and the 128-B record layouts."""
    n, d = 3000, 256
    base = graphs.features(n, d, seed=k)
    special = _stat_rows(16, d, seed=k + 1)
    for r in [None] + list(range(3, 10)):
        x = base.clone()
        if r is not None:
            x[1234] = special[r]
        xd = x.to(gpu)
        if records:
            rb = max(128, -(-5 * k // 16) * 16)
            rec = torch.empty((n, rb), dtype=torch.uint8, device=gpu)
            sd, si = rec[:, :4 * k].view(torch.float32), rec[:, 4 * k:5 * k]
            if k % 4:
                pytest.skip("records need k % 4 == 0")
        else:
            sd = torch.empty((n, k), device=gpu)
            si = torch.empty((n, k), dtype=torch.uint8, device=gpu)
        st = torch.empty(2, dtype=torch.int32, device=gpu).fill_(-1)
        mk.maxk_forward(xd, k, mode=mode, return_index=True, out=(sd, si), stats=st)
        ref = mk.cbsr_stats(sd, si)
        assert st.tolist() == ref.view(-1).tolist(), (r, st.tolist(), ref.tolist())
        d0, i0 = mk.maxk_forward(xd, k, mode=mode, return_index=True)
        assert torch.equal(si.cpu(), i0.cpu())
        assert np.array_equal(sd.cpu().numpy().view(np.uint32), d0.cpu().numpy().view(np.uint32))


def test_topk_fused_stats_empty_and_tiny(gpu):
    """N = 0 writes the all-zero pair (the forward then takes f64); N = 1 and N = 5."""
    st = torch.empty(2, dtype=torch.int32, device=gpu).fill_(7)
    x = torch.empty((0, 64), device=gpu)
    mk.maxk_forward(x, 8, return_index=True, stats=st)
    assert st.tolist() == [0, 0]
    for n in (1, 5):
        x = graphs.features(n, 64, seed=n).to(gpu)
        sd, si = mk.maxk_forward(x, 8, return_index=True, stats=st)
        assert st.tolist() == mk.cbsr_stats(sd, si).view(-1).tolist()
    with pytest.raises(RuntimeError, match="stats must be"):
        mk.maxk_forward(x, 8, return_index=True, stats=torch.empty(3, dtype=torch.int32,
                                                                   device=gpu))


@pytest.mark.parametrize("k", [8, 16, 24, 32, 64])
@pytest.mark.parametrize("mode", ["exact", "ref_compat"])
def test_maxk_aggregate_fused_equals_unfused(gpu, k, mode):
    """maxk_aggregate (top-k writing the forward's layout and statistics, no pack or statistics
    pass) against MaxKFunction -> SpGEMMFunction and the oracle: the output equals the unfused
    one bitwise where the forward is fixed point (k >= 16: integer sums, the same statistics);
    both outputs and both input gradients within the oracle bound (the backward's f32 LDS
    accumulation order varies from run to run); plan layouts covered: lane chunks (k = 8, 24),
    pair chunks (16), two tables (32, 64)."""
    pt, it = graphs.synthetic_csr(2000, 300_000, seed=37)   # 150 edges per column: k = 16
    p, ix, v = pt.numpy(), it.numpy(), graphs.sage_mean_values(pt).numpy()  # packs records
    n, d = p.size - 1, 256
    x = graphs.features(n, d, seed=31 + k)
    x[::7, 5] = 1e6                          # ref_compat: single-hit rows with padding slots
    g = graphs.features(n, d, seed=32 + k).to(gpu)
    graph = mk.CSRGraph(*graph_on(gpu, p, ix, v))
    layout = graph.plan(d, k).info()["fwd_layout"]
    assert layout == {8: 2, 24: 2, 16: 4, 32: 0, 64: 0}[k]
    x1 = x.to(gpu).requires_grad_(True)
    y1 = mk.maxk_aggregate(x1, graph, k, mode)
    y1.backward(g)
    x2 = x.to(gpu).requires_grad_(True)
    sd, si = mk.maxk(x2, k, mode)
    y2 = mk.spgemm(sd, si, graph, d)
    y2.backward(g)
    if k >= 16:
        assert torch.equal(y1, y2)
    od, oi = oracle.maxk(x.numpy(), k, mode)
    ref, mag = oracle.spgemm_forward(p, ix, v, od, oi, d, with_mag=True)
    assert_close(y1, ref, mag)
    assert_close(y2, ref, mag)
    gs, gmag = oracle.sspmm_backward(p, ix, v, g.cpu().numpy(), oi, with_mag=True)
    filled = od != 0 if mode == "ref_compat" else np.ones_like(od, bool)
    gx_ref = np.zeros((n, d))
    gx_mag = np.zeros((n, d))
    rows = np.repeat(np.arange(n)[:, None], k, 1)
    gx_ref[rows[filled], oi[filled]] = gs[filled]      # ascending unique selectors per row
    gx_mag[rows[filled], oi[filled]] = gmag[filled]
    assert_close(x1.grad, gx_ref, gx_mag)
    assert_close(x2.grad, gx_ref, gx_mag)


# ------------------------------------------------ the reference's own layer code, unchanged
def test_reference_layer_call_sequences(gpu):
    """With this package first on PYTHONPATH, the reference's unchanged training script
    (maxk_gnn_integrated.py:21 -> utils/integrated_models.py:6 -> utils/maxk_layers.py:10
    `import maxk_kernels`) calls these functions exactly as below, with the argument types that
    code builds (replayed here; the reference itself, which needs DGL, is not imported):

    * maxk_layers.py:21   maxk_forward(input, k) -> [N, k] f32 values;
    * maxk_layers.py:23,40 maxk_backward(grad [N, k], torch.topk(input, k)[1] int64, unsorted)
      -> [N, max(index) + 1];
    * maxk_layers.py:166-171 (SAGE) spgemm_forward(ptr.int(), idx.int(), f32 weights from a
      Python list, torch.stack of f32 rows, torch.stack of u8 rows, N, E, maxk, out_feats)
      -> (out, sp_index), out against the oracle;
    * maxk_layers.py:380-385 (GCN) spgemm_forward with DGL's int64 adj_tensors: refused with
      the reference binding's message (bindings.cpp:45-54 checks int32), as there."""
    p, ix, v = GRAPHS["synthetic"]()
    n, d, k = p.size - 1, 64, 16
    x = graphs.features(n, d, seed=71).to(gpu)
    out = mk.maxk_forward(x, k)                                    # :21
    assert out.shape == (n, k) and out.dtype == torch.float32
    od, oi = oracle.maxk(x.cpu().numpy(), k)
    assert np.array_equal(out.cpu().numpy(), od)
    indices = torch.topk(x, k, dim=1)[1]                           # :23, int64, value order
    g = torch.randn(n, k, device=gpu)
    gi = mk.maxk_backward(g, indices)                              # :40
    width = int(indices.max()) + 1
    ref = np.zeros((n, width), np.float32)
    ind = indices.cpu().numpy()
    for j in range(k):                                             # last slot wins
        ref[np.arange(n), ind[:, j]] = g.cpu().numpy()[:, j]
    assert gi.shape == (n, width) and np.array_equal(gi.cpu().numpy(), ref)
    # SAGE aggregation as _aggregate_with_custom_kernel builds its arguments
    ptr, idx = torch.from_numpy(p).long().to(gpu), torch.from_numpy(ix).long().to(gpu)
    deg = np.diff(p)
    w = torch.tensor([1.0 / max(int(c), 1) for c in deg for _ in range(int(c))], device=gpu)
    sp_data = torch.stack([out[i] for i in range(n)])              # :233-262, contiguous
    sp_index = torch.stack([torch.from_numpy(oi[i]).to(gpu) for i in range(n)])
    agg, si = mk.spgemm_forward(ptr.int(), idx.int(), w, sp_data, sp_index, n, ix.size, k, d)
    assert si is sp_index
    yref, ymag = oracle.spgemm_forward(p, ix, w.cpu().numpy(), od, oi, d, with_mag=True)
    assert_close(agg, yref, ymag)
    # GCN: DGL's adj_tensors('csr') are int64; the reference binding requires int32
    with pytest.raises(RuntimeError, match="ptr must be int32"):
        mk.spgemm_forward(ptr, idx, w, sp_data, sp_index, n, ix.size, k, d)
