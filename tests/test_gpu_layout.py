"""GPU: the ABI-2 layout options against the oracle.

* column orders of the backward's column blocks (identity / scattered / the caller's
  permutation, checked through the raw C ABI against the header's documented values) and the
  row order of the block streams, on graphs with and without community structure in ID
  order;
* row chunks of the two-pass backward (bounded workspace);
* the fixed-point forward's bound with repeated selectors (maxk_hip.h: repeated selectors in
  one CBSR row are summed) and the per-part statistics of maxk_spgemm_forward_ex;
* the dense comparator at hidden sizes that are not a multiple of 4;
* maxk_plan_get_info writes only the version-1 struct.
"""
import ctypes

import numpy as np
import pytest
import torch

import maxk_kernels as mk
from maxk_kernels import _lib, graphs
from oracle import oracle

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def assert_close(got, ref, mag, rtol=RTOL):
    got = got.detach().cpu().numpy() if torch.is_tensor(got) else got
    ok, worst = oracle.close_enough(got, ref, mag, rtol=rtol)
    assert ok, f"worst err/bound = {worst:.3g}"


def community(n=12_000, e=600_000, shuffle=False, seed=71):
    p, i = graphs.community_csr(n, e, communities=9, seed=seed, shuffle=shuffle)
    return p.numpy(), i.numpy(), graphs.gcn_values(p, i).numpy()


_GRAPHS = {}


def graph(name):
    if name not in _GRAPHS:
        if name == "uniform":
            p, i = graphs.synthetic_csr(12_000, 600_000, seed=72)
            _GRAPHS[name] = (p.numpy(), i.numpy(), graphs.sage_mean_values(p).numpy())
        else:
            _GRAPHS[name] = community(shuffle=name == "community_shuffled")
    return _GRAPHS[name]


def dev(a, gpu):
    return torch.from_numpy(np.ascontiguousarray(a)).to(gpu)


@pytest.mark.parametrize("gname", ["uniform", "community", "community_shuffled"])
@pytest.mark.parametrize("order", ["identity", "scattered", "given"])
@pytest.mark.parametrize("k", [8, 16, 32])
@pytest.mark.parametrize("rows", [1, 2])
def test_col_order_and_row_order_vs_oracle(gpu, gname, order, k, rows):
    p, ix, v = graph(gname)
    n, d = p.size - 1, 256
    x = graphs.features(n, d, seed=k)
    g = graphs.features(n, d, seed=k + 1)
    od, oi = oracle.maxk(x.numpy(), k)
    ref_f, mag_f = oracle.spgemm_forward(p, ix, v, od, oi, d, with_mag=True)
    ref_b, mag_b = oracle.sspmm_backward(p, ix, v, g.numpy(), oi, with_mag=True)
    opts = dict(bwd_row_order=rows, bwd_tasks_per_cu=8, bwd_min_task_edges=2000)
    perm = None
    if order == "given":
        perm = torch.from_numpy(np.random.RandomState(k).permutation(n).astype(np.int32)).to(gpu)
    else:
        opts["col_order"] = order
    plan = mk.GraphPlan(dev(p, gpu), dev(ix, gpu), dev(v, gpu), n, ix.size, d, k, options=opts,
                        col_order=perm)
    info = plan.info()
    assert info["bwd_row_order"] == rows
    assert info["col_order"] == _lib.COL_ORDERS[order]
    assert info["bwd_chunk_bounds"] == 2
    if perm is not None:
        assert torch.equal(mk.plan_col_order(plan), perm)
    assert_close(plan.forward(dev(od, gpu), dev(oi, gpu)), ref_f, mag_f)
    gs = plan.backward(g.to(gpu), dev(oi, gpu))
    assert_close(gs, ref_b, mag_b)
    # every element written (the slab flush stores zero blocks too)
    again = torch.full_like(gs, float("nan"))
    plan.backward(g.to(gpu), dev(oi, gpu), again)
    torch.cuda.synchronize()
    assert not torch.isnan(again).any()
    assert_close(again, ref_b, mag_b)


def _header_enum(prefix):
    import os
    import re
    text = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                             "include", "maxk_hip.h")).read()
    return {m.group(1): int(m.group(2))
            for m in re.finditer(r"\b(" + prefix + r"\w+)\s*=\s*(\d+)", text)}


@pytest.mark.parametrize("mode", ["MAXK_COL_ORDER_AUTO", "MAXK_COL_ORDER_IDENTITY",
                                  "MAXK_COL_ORDER_SCATTERED", "MAXK_COL_ORDER_GIVEN"])
def test_capi_col_order_info_matches_header(gpu, mode):
    """maxk_plan_create_sized with each documented col_order value, straight through the C
    ABI: maxk_plan_info.col_order reads back the header's enumeration (auto = identity), and
    maxk_plan_get_col_order returns the order the blocks use."""
    enum = _header_enum("MAXK_COL_ORDER_")
    p, ix, v = graph("uniform")
    n, d, k = p.size - 1, 256, 16
    dp, di, dv = dev(p, gpu), dev(ix, gpu), dev(v, gpu)
    opts = _lib.PlanOptions()
    opts.col_order = enum[mode]
    perm = torch.from_numpy(np.random.RandomState(3).permutation(n).astype(np.int32)).to(gpu)
    h = ctypes.c_void_p(0)
    P = ctypes.c_void_p
    rc = _lib.lib.maxk_plan_create_sized(P(dp.data_ptr()), P(di.data_ptr()), P(dv.data_ptr()),
                                         n, n, ix.size, d, k, ctypes.byref(opts),
                                         ctypes.sizeof(opts),
                                         P(perm.data_ptr()) if mode.endswith("GIVEN") else None,
                                         P(torch.cuda.current_stream().cuda_stream),
                                         ctypes.byref(h))
    assert rc == 0, _lib.lib.maxk_last_error()
    try:
        info = _lib.PlanInfo()
        assert _lib.lib.maxk_plan_get_info_sized(h, ctypes.byref(info), ctypes.sizeof(info)) == 0
        want = enum["MAXK_COL_ORDER_IDENTITY"] if mode.endswith("AUTO") else enum[mode]
        assert info.col_order == want
        assert info.bwd_algo == _header_enum("MAXK_BWD_")["MAXK_BWD_COLUMN_BLOCKS"]
        got = torch.empty(n, dtype=torch.int32, device=gpu)
        assert _lib.lib.maxk_plan_get_col_order(h, P(got.data_ptr()),
                                                P(torch.cuda.current_stream().cuda_stream)) == 0
        torch.cuda.synchronize()
        if mode.endswith("GIVEN"):
            assert torch.equal(got, perm)
        elif mode.endswith("SCATTERED"):
            assert torch.equal(torch.sort(got.long()).values, torch.arange(n, device=gpu))
            assert not torch.equal(got.long(), torch.arange(n, device=gpu))
        else:
            assert torch.equal(got.long(), torch.arange(n, device=gpu))
    finally:
        _lib.lib.maxk_plan_destroy(h)


def test_given_col_order(gpu):
    p, ix, v = graph("community")
    n, d, k = p.size - 1, 256, 16
    g = graphs.features(n, d, seed=3)
    _, oi = oracle.maxk(graphs.features(n, d, seed=2).numpy(), k)
    ref, mag = oracle.sspmm_backward(p, ix, v, g.numpy(), oi, with_mag=True)
    perm = torch.from_numpy(np.random.RandomState(5).permutation(n).astype(np.int32)).to(gpu)
    plan = mk.GraphPlan(dev(p, gpu), dev(ix, gpu), dev(v, gpu), n, ix.size, d, k,
                        col_order=perm)
    assert plan.info()["col_order"] == 4
    assert_close(plan.backward(g.to(gpu), dev(oi, gpu)), ref, mag)
    got = mk.plan_col_order(plan)
    assert torch.equal(got, perm)
    # not a permutation: a repeat, and entries outside [0, n) far beyond the buffer (refused
    # on the host before any device scatter uses them)
    for bad_value in ("repeat", n, -1, 1 << 30, -(1 << 30)):
        bad = perm.clone()
        bad[7] = bad[8] if bad_value == "repeat" else bad_value
        with pytest.raises(RuntimeError, match="permutation"):
            mk.GraphPlan(dev(p, gpu), dev(ix, gpu), dev(v, gpu), n, ix.size, d, k, col_order=bad)
    # the device is still healthy and the good order still works
    again = mk.GraphPlan(dev(p, gpu), dev(ix, gpu), dev(v, gpu), n, ix.size, d, k, col_order=perm)
    assert_close(again.backward(g.to(gpu), dev(oi, gpu)), ref, mag)


@pytest.mark.parametrize("chunks", [1, 2, 7])
@pytest.mark.parametrize("k", [16, 32])
def test_twopass_row_chunks(gpu, chunks, k):
    p, ix, v = graph("uniform")
    n, d = p.size - 1, 256
    g = graphs.features(n, d, seed=11)
    _, oi = oracle.maxk(graphs.features(n, d, seed=12).numpy(), k)
    ref, mag = oracle.sspmm_backward(p, ix, v, g.numpy(), oi, with_mag=True)
    plan = mk.GraphPlan(dev(p, gpu), dev(ix, gpu), dev(v, gpu), n, ix.size, d, k,
                        options=dict(bwd_algo=3, bwd_tp_chunks=chunks))
    info = plan.info()
    assert info["bwd_algo"] == 3 and info["bwd_tp_chunks"] == chunks
    # the workspace holds the largest chunk's products
    assert info["bwd_workspace_peak"] <= (ix.size // chunks + np.diff(p).max()) * k * 4
    assert_close(plan.backward(g.to(gpu), dev(oi, gpu)), ref, mag)
    v2 = dev(v * np.float32(-0.5), gpu)
    plan.refresh_values(v2)
    ref2, mag2 = oracle.sspmm_backward(p, ix, v * np.float32(-0.5), g.numpy(), oi, with_mag=True)
    assert_close(plan.backward(g.to(gpu), dev(oi, gpu)), ref2, mag2)


@pytest.mark.parametrize("k", [16, 32])
@pytest.mark.parametrize("pattern", ["all_same", "pairs", "one_row"])
def test_fixed_point_repeated_selectors(gpu, k, pattern):
    """Rows whose nonzero entries repeat a selector add several terms to one LDS slot. The
    fixed-point bound must cover the sum (a max |x| bound let k near-maximal terms reach
    2^52 and wrap the 51-bit residue): forced fixed point against the oracle."""
    ptr, idx = graphs.synthetic_csr(4000, 200_000, seed=74)
    p, ix = ptr.numpy(), idx.numpy()
    v = np.random.RandomState(74).uniform(0.5, 1.0, ix.size).astype(np.float32)
    n, d = p.size - 1, 256
    od, oi = oracle.maxk(graphs.features(n, d, seed=75).numpy(), k)
    od = np.abs(od).astype(np.float32)
    big = np.float32(1.0 - 2.0 ** -20)
    if pattern == "all_same":
        oi[:] = 5
        od[:] = big
    elif pattern == "pairs":
        oi[:, 1::2] = oi[:, 0::2]
        od[:, :2] = big
    else:
        oi[17, :] = 200
        od[17, :] = big
    ref, mag = oracle.spgemm_forward(p, ix, v, od, oi, d, with_mag=True)
    plan = mk.GraphPlan(dev(p, gpu), dev(ix, gpu), dev(v, gpu), n, ix.size, d, k,
                        options=dict(fwd_fixed=1))
    assert_close(plan.forward(dev(od, gpu), dev(oi, gpu)), ref, mag)


def _stats_numpy(od, oi):
    """maxk_cbsr_stats restated: per row max |x|, or the sum when nonzero selectors do not
    strictly ascend; the min nonzero |x|."""
    a = np.abs(od)
    mx, mn = 0.0, np.inf
    for r in range(a.shape[0]):
        nz = a[r] != 0
        if not nz.any():
            continue
        s = oi[r][nz].astype(np.int64)
        rep = bool((np.diff(s) <= 0).any())
        acc = np.float32(0.0)
        for t in a[r][nz]:                   # the kernel's sequential f32 sum
            acc = np.float32(acc + np.float32(t))
        b = np.float32(acc * np.float32(1 + 2.0 ** -10)) if rep else a[r].max()
        mx = max(mx, float(max(b, a[r].max())))
        mn = min(mn, float(a[r][nz].min()))
    return mx, mn


def test_cbsr_stats_and_forward_ex_split(gpu):
    ptr, idx = graphs.synthetic_csr(3000, 90_000, seed=76)
    p, ix = ptr.numpy(), idx.numpy()
    v = graphs.sage_mean_values(ptr).numpy()
    n, d, k = p.size - 1, 256, 16
    od, oi = oracle.maxk(graphs.features(n, d, seed=77).numpy(), k)
    od, oi = od.copy(), oi.copy()
    oi[9, 3] = oi[9, 2]                      # one row with a repeated selector
    od[10, :] = 0.0                          # an empty row
    st = mk.cbsr_stats(dev(od, gpu), dev(oi, gpu)).cpu().numpy().view(np.uint32)[0]
    mx, mn = _stats_numpy(od, oi)
    # the repeated row's bound is its f32 sum of |x| (+2^-10), summed in the kernel's order
    got = float(np.uint32(st[0]).view(np.float32))
    assert mx * (1 - 2.0 ** -20) <= got <= mx * (1 + 2.0 ** -20)
    assert st[1] == 0x7FFFFFFF - np.float32(mn).view(np.uint32)
    # without the repeat the bound is exactly the max |x|
    oi2 = oracle.maxk(graphs.features(n, d, seed=77).numpy(), k)[1]
    st2 = mk.cbsr_stats(dev(od, gpu), dev(oi2, gpu)).cpu().numpy().view(np.uint32)[0]
    assert st2[0] == np.abs(od).max().view(np.uint32)
    # the stats of two halves of the table, as the multi-GPU path gathers them per rank
    sd, si = dev(od, gpu), dev(oi, gpu)
    halves = torch.cat([mk.cbsr_stats(sd[:1500], si[:1500]), mk.cbsr_stats(sd[1500:], si[1500:])])
    plan = mk.GraphPlan(dev(p, gpu), dev(ix, gpu), dev(v, gpu), n, ix.size, d, k,
                        options=dict(fwd_fixed=1))
    a = plan.forward(sd, si)
    b = plan.forward(sd, si, stats=halves)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    ref, mag = oracle.spgemm_forward(p, ix, v, od, oi, d, with_mag=True)
    assert_close(b, ref, mag)


@pytest.mark.parametrize("width", [30, 66, 7, 512, 1000])
def test_dense_spmm_any_width(gpu, width):
    ptr, idx = graphs.synthetic_csr(2000, 40_000, seed=78)
    p, ix = ptr.numpy(), idx.numpy()
    v = graphs.sage_mean_values(ptr).numpy()
    x = graphs.features(2000, width, seed=79)
    ref = oracle.dense_spmm(p, ix, v, x.numpy())
    mag = oracle.dense_spmm(p, ix, np.abs(v), np.abs(x.numpy()))
    y = mk.dense_spmm(dev(p, gpu), dev(ix, gpu), dev(v, gpu), x.to(gpu))
    assert y.shape == (2000, width)
    assert_close(y, ref, mag, rtol=2e-6 * 64)


def test_get_info_v1_writes_only_v1_fields(gpu):
    p, ix, v = graph("uniform")
    plan = mk.GraphPlan(dev(p, gpu), dev(ix, gpu), dev(v, gpu), p.size - 1, ix.size, 256, 16)
    buf = (ctypes.c_uint8 * ctypes.sizeof(_lib.PlanInfo))(*([0xAB] * ctypes.sizeof(_lib.PlanInfo)))
    assert _lib.lib.maxk_plan_get_info(plan.handle, ctypes.cast(buf, ctypes.c_void_p)) == 0
    v1 = _lib.PlanInfo.col_order.offset
    assert all(b == 0xAB for b in bytes(buf)[v1:])
    info = _lib.PlanInfo.from_buffer_copy(bytes(buf))
    assert info.num_edges == ix.size and info.bwd_algo in (1, 2, 3)


def test_auto_row_order_follows_dense_runs(gpu):
    """bwd_row_order auto: scattered rows only where the ascending-row block streams are
    mostly dense runs (an ID-ordered community graph), ascending elsewhere."""
    expect = {"uniform": 1, "community": 2, "community_shuffled": 1}
    for name, want in expect.items():
        p, ix, v = graph(name)
        plan = mk.GraphPlan(dev(p, gpu), dev(ix, gpu), dev(v, gpu), p.size - 1, ix.size, 256, 16)
        assert plan.info()["bwd_row_order"] == want, name


@pytest.mark.parametrize("k", [8, 16, 12, 20, 10])
def test_cbsr_stats_repeat_detection(gpu, k):
    """A repeated selector is found whatever lies between the two entries (zeros, other lanes'
    entries); zero padding after the filled slots (ref_compat rows) is not a repeat."""
    base = np.arange(1, k + 1, dtype=np.int64) * 3
    cases = []
    s = base.copy(); s[2] = s[0]; cases.append((s, np.ones(k), True))            # same lane
    s = base.copy(); s[k - 1] = s[0]; cases.append((s, np.ones(k), True))        # far lanes
    s = base.copy(); s[1] = 1; s[2] = s[0]; x = np.ones(k); x[1] = 0.0           # zero between
    cases.append((s, x, True))
    s = base.copy(); s[k // 2:] = 0; x = np.ones(k); x[k // 2:] = 0.0            # padding
    cases.append((s, x, False))
    cases.append((base.copy(), np.ones(k), False))                              # ascending
    for s, x, rep in cases:
        xs = (x * np.linspace(1.0, 2.0, k)).astype(np.float32)[None, :]
        st = mk.cbsr_stats(dev(xs, gpu), dev(s.astype(np.uint8)[None, :], gpu))
        got = float(np.uint32(st.cpu().numpy().view(np.uint32)[0, 0]).view(np.float32))
        want = xs.sum() * (1 + 2.0 ** -10) if rep else xs.max()
        assert abs(got - want) <= 1e-6 * want, (k, s, x, got, want)


@pytest.mark.parametrize("k", [8, 16])
def test_skewed_column_blocks_keep_their_chunks(gpu, k):
    """the chunk-count search may go below the nominal chunk count only while the
    column blocks hold similar edge counts. A graph whose in-edges pile onto the first columns
    (power-law source degrees, Zipf-like) has one block many times the mean: the plan keeps at
    least the nominal task count (one round of CUs or more, every block cut into the same
    number of chunks) and the backward matches the oracle."""
    n, e = 120_000, 4_000_000
    rs = np.random.RandomState(5)
    deg = np.minimum(rs.lognormal(np.log(e / n) - 0.5, 1.0, n).astype(np.int64) + 1, n)
    scale = e / deg.sum()
    deg = np.maximum(1, (deg * scale).astype(np.int64))
    ptr = np.zeros(n + 1, np.int64)
    ptr[1:] = np.cumsum(deg)
    cols = np.minimum((rs.pareto(0.7, int(ptr[-1])) * 50).astype(np.int64), n - 1)
    idx = np.concatenate([np.sort(cols[ptr[r]:ptr[r + 1]]) for r in range(n)]).astype(np.int32)
    ptr = ptr.astype(np.int32)
    val = rs.uniform(0.1, 1.0, idx.size).astype(np.float32)
    dptr, didx, dval = (torch.from_numpy(a).to(gpu) for a in (ptr, idx, val))
    plan = mk.GraphPlan(dptr, didx, dval, n, idx.size, 256, k, options={"bwd_algo": 1})
    info = plan.info()
    counts = np.bincount(idx, minlength=n)
    cb = info["bwd_block_cols"]
    per_block = np.add.reduceat(counts, np.arange(0, n, cb))
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    print(f"k={k}: {info['bwd_blocks']} blocks, largest {per_block.max()} edges vs mean "
          f"{per_block.mean():.0f}; {info['bwd_tasks']} tasks on {cus} CUs")
    assert per_block.max() > 2 * per_block.mean()           # the case the bound is for
    assert info["bwd_tasks"] >= min(cus, info["bwd_blocks"])
    x = graphs.features(n, 256, seed=k)
    _, oi = oracle.maxk(x.numpy(), k)
    g = graphs.features(n, 256, seed=k + 1)
    gs = plan.backward(g.to(gpu), torch.from_numpy(oi).to(gpu))
    ref, mag = oracle.sspmm_backward(ptr, idx, val, g.numpy(), oi, with_mag=True)
    ok, worst = oracle.close_enough(gs.cpu().numpy(), ref, mag)
    assert ok, worst
