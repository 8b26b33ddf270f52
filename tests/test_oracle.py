"""CPU: the oracle against independent formulations and against the committed fixtures.

The reference has no tests or golden vectors for this path, so the oracle is
pinned two ways: (1) independent torch / pure-Python formulations of each decoded
semantic (SURVEY §8(c) "independent torch formulations"), (2) tests/golden/maxk_small.npz.
"""
import os

import numpy as np
import pytest
import torch

from oracle import oracle
from maxk_kernels import graphs

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "maxk_small.npz")


@pytest.fixture(scope="module")
def golden():
    with np.load(GOLDEN, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def small_graph(n=300, e=6000, seed=5):
    ptr, idx = graphs.synthetic_csr(n, e, seed=seed)
    val = graphs.sage_mean_values(ptr)
    return ptr, idx, val


def densify(data, index, d):
    n, k = data.shape
    x = torch.zeros(n, d, dtype=torch.float64)
    x.scatter_add_(1, torch.as_tensor(index, dtype=torch.int64),
                   torch.as_tensor(data, dtype=torch.float64))
    return x


def ref_compat_py(row, k):
    """Literal pure-Python restatement of SURVEY §8 a1 (thread 0 of maxk_kernel), f32."""
    f = np.float32
    s = [f(v) for v in row]
    lo = hi = s[0]
    for v in s[1:]:  # FMNMX: a NaN operand yields the other one (np.fmin / np.fmax)
        lo = f(np.fmin(lo, v))
        hi = f(np.fmax(hi, v))
    p = f(f(lo + hi) * f(0.5))
    for _ in range(8):
        cnt = sum(1 for v in s if v > p)
        if cnt == k:
            break
        if cnt >= k:
            lo = p
        else:
            hi = p
        p = f(f(lo + hi) * f(0.5))
    data, index = [], []
    for i, v in enumerate(s):
        if v > p:
            data.append(v)
            index.append(i)
            if len(data) >= k:
                break
    data += [f(0)] * (k - len(data))
    index += [0] * (k - len(index))
    return np.array(data, np.float32), np.array(index, np.uint8)


@pytest.mark.parametrize("k", [1, 8, 16, 24, 32, 64, 256])
def test_exact_topk_matches_torch(k):
    x = torch.randn(200, 256, generator=torch.Generator().manual_seed(k))
    d, i = oracle.maxk(x.numpy(), k, "exact")
    ti = torch.topk(x, k, dim=1).indices.sort(dim=1).values
    assert np.array_equal(i.astype(np.int64), ti.numpy())
    assert np.array_equal(d, torch.gather(x, 1, ti).numpy())


def test_exact_topk_ties_lowest_index():
    x = np.zeros((3, 64), np.float32)
    x[0, :] = 1.0                           # all tied -> first k
    x[1, :] = np.arange(64) % 4             # ties at the threshold value 3 (16 copies)
    x[2, 10:20] = 5.0
    d, i = oracle.maxk(x, 8, "exact")
    assert list(i[0]) == list(range(8))
    assert list(i[1]) == [3, 7, 11, 15, 19, 23, 27, 31]
    assert list(i[2]) == list(range(10, 18))


@pytest.mark.parametrize("k", [4, 16, 32, 100])
def test_ref_compat_matches_python_restatement(k):
    x = np.random.RandomState(k).randn(40, 256).astype(np.float32)
    x[0, :] = 2.0
    d, i = oracle.maxk(x, k, "ref_compat")
    for r in range(x.shape[0]):
        pd, pi = ref_compat_py(x[r], k)
        assert np.array_equal(pd, d[r]) and np.array_equal(pi, i[r]), r


NAN_ROWS = os.path.join(os.path.dirname(__file__), "golden", "maxk_exact_nan.npz")


def _torch_key(x):
    """torch.topk's radix key (every NaN -> the largest key, all NaNs equal)."""
    b = x.view(np.uint32).astype(np.uint64)
    key = np.where(b & 0x80000000, ~b & 0xffffffff, b | 0x80000000)
    return np.where((b & 0x7fffffff) > 0x7f800000, 0xffffffff, key)


@pytest.mark.parametrize("k", [1, 8, 16, 32, 64])
def test_exact_nan_order_matches_torch_topk(k):
    """Exact mode ranks every NaN, either sign and any payload, above +Inf (torch.topk,
    utils/models.py:15): the committed fixture equals the oracle bit for bit, and each row's
    index set is torch.topk's wherever the k-th and (k+1)-th keys differ; where they tie (NaN
    ties included), the selected keys are torch's and the tie goes to the lowest indices."""
    with np.load(NAN_ROWS, allow_pickle=False) as z:
        x, gd, gi = z["x"], z[f"data_k{k}"], z[f"index_k{k}"]
    d, i = oracle.maxk(x, k, "exact")
    assert np.array_equal(i, gi) and np.array_equal(d.view(np.uint32), gd.view(np.uint32))
    ti = torch.topk(torch.from_numpy(x), k, dim=1).indices.numpy()
    nan_rows = 0
    for r in range(x.shape[0]):
        key = _torch_key(x[r])
        order = np.argsort(-key.astype(np.float64), kind="stable")   # ties: lowest index first
        assert sorted(order[:k]) == list(gi[r]), r
        assert np.array_equal(d[r].view(np.uint32), x[r][gi[r]].view(np.uint32)), r
        # CPU torch.topk compares values, so +0 and -0 tie there (its GPU radix keys order them)
        with np.errstate(invalid="ignore"):
            ck = _torch_key(x[r] + np.float32(0.0))
        assert sorted(ck[ti[r]]) == sorted(ck[gi[r]]), r                 # same keys as torch
        if k < x.shape[1] and ck[order[k - 1]] != ck[order[k]]:
            assert set(ti[r]) == set(gi[r]), r                         # no tie: same set
        nan_rows += bool(np.isnan(x[r][gi[r]]).any())
    assert nan_rows == x.shape[0]             # every row holds a NaN, so every row selects one


EDGE = os.path.join(os.path.dirname(__file__), "golden", "maxk_refcompat_edge.npz")


@pytest.mark.parametrize("k", [1, 8, 16, 32, 64])
def test_ref_compat_edge_fixtures(k):
    """NaN / +-Inf / +-0 / all-equal / cap-with-cnt>k / cap-with-cnt<k / denormal rows
    (tests/golden/make_golden.py:edge_rows): the committed fixture, the C oracle and the
    literal restatement agree bit for bit."""
    with np.load(EDGE, allow_pickle=False) as z:
        x, gd, gi = z["x"], z[f"data_k{k}"], z[f"index_k{k}"]
    d, i = oracle.maxk(x, k, "ref_compat")
    assert np.array_equal(i, gi) and np.array_equal(d.view(np.uint32), gd.view(np.uint32))
    with np.errstate(invalid="ignore", over="ignore"):
        for r in range(x.shape[0]):
            pd, pi = ref_compat_py(x[r], k)
            assert np.array_equal(pi, gi[r]), r
            assert np.array_equal(pd.view(np.uint32), gd[r].view(np.uint32)), r


def test_ref_compat_edge_fixtures_cover_the_cap_exits():
    """The fixture holds a row ending the 8 steps with cnt > k (k slots filled from more
    candidates) and one with cnt < k (padding (0.0f, 0) after the last hit)."""
    with np.load(EDGE, allow_pickle=False) as z:
        x, gi = z["x"], z["index_k16"]
    k = 16
    counts = []
    for r in range(x.shape[0]):
        pd, pi = ref_compat_py(x[r], k)
        counts.append(int((pd != 0).sum()))
    assert counts[10] == k and (x[10] > 0).sum() > k  # cnt > k at the cap
    assert 0 < counts[11] < k                          # cnt < k at the cap


@pytest.mark.parametrize("k", [8, 16, 24, 64])
def test_spgemm_forward_matches_torch_sparse(k):
    ptr, idx, val = small_graph()
    n = ptr.numel() - 1
    x = torch.randn(n, 128, generator=torch.Generator().manual_seed(1))
    d, i = oracle.maxk(x.numpy(), k)
    y, mag = oracle.spgemm_forward(ptr.numpy(), idx.numpy(), val.numpy(), d, i, 128,
                                   with_mag=True)
    a = torch.sparse_csr_tensor(ptr.long(), idx.long(), val.double(), size=(n, n))
    ref = (a @ densify(d, i, 128)).numpy()
    ok, worst = oracle.close_enough(y, ref, mag, rtol=1e-6)
    assert ok, worst


def test_spgemm_forward_sums_duplicate_selectors():
    ptr = np.array([0, 2, 3], np.int32)
    idx = np.array([0, 1, 1], np.int32)
    val = np.array([1.0, 2.0, 0.5], np.float32)
    data = np.array([[1.0, 10.0], [3.0, 4.0]], np.float32)
    index = np.array([[5, 5], [0, 7]], np.uint8)   # row 0 repeats selector 5
    y = oracle.spgemm_forward(ptr, idx, val, data, index, 8)
    assert y[0, 5] == 11.0 and y[0, 0] == 6.0 and y[0, 7] == 8.0
    assert y[1, 0] == 1.5 and y[1, 7] == 2.0


@pytest.mark.parametrize("k", [8, 16, 32])
def test_sspmm_backward_is_sampled_AT_G(k):
    ptr, idx, val = small_graph(seed=9)
    n = ptr.numel() - 1
    x = torch.randn(n, 64, generator=torch.Generator().manual_seed(2))
    g = torch.randn(n, 64, generator=torch.Generator().manual_seed(3))
    _, i = oracle.maxk(x.numpy(), k)
    gs, mag = oracle.sspmm_backward(ptr.numpy(), idx.numpy(), val.numpy(), g.numpy(), i,
                                    with_mag=True)
    a = torch.sparse_csr_tensor(ptr.long(), idx.long(), val.double(), size=(n, n))
    at_g = (a.to_dense().t() @ g.double())
    ref = at_g.gather(1, torch.as_tensor(i, dtype=torch.int64)).numpy()
    ok, worst = oracle.close_enough(gs, ref, mag, rtol=1e-6)
    assert ok, worst


def test_forward_backward_adjoint():
    """<A densify(sp), G> == <sp_data, grad_sp>: the SSpMM is the SpGEMM's adjoint."""
    ptr, idx, val = small_graph(seed=11)
    n = ptr.numel() - 1
    x = np.random.RandomState(4).randn(n, 64).astype(np.float32)
    g = np.random.RandomState(5).randn(n, 64).astype(np.float32)
    d, i = oracle.maxk(x, 16)
    y = oracle.spgemm_forward(ptr.numpy(), idx.numpy(), val.numpy(), d, i, 64)
    gs = oracle.sspmm_backward(ptr.numpy(), idx.numpy(), val.numpy(), g, i)
    lhs = float((y.astype(np.float64) * g).sum())
    rhs = float((d.astype(np.float64) * gs).sum())
    assert abs(lhs - rhs) <= 1e-5 * (abs(lhs) + 1)


def test_maxk_backward_slot_order_assignment():
    grad = np.array([[1.0, 2.0, 3.0]], np.float32)
    index = np.array([[4, 1, 4]], np.uint8)  # repeated index: the last slot wins
    out = oracle.maxk_backward(grad, index, 6)
    assert list(out[0]) == [0.0, 2.0, 0.0, 0.0, 3.0, 0.0]


def test_dense_spmm_mean_matches_torch():
    ptr, idx, _ = small_graph(seed=13)
    n = ptr.numel() - 1
    x = np.random.RandomState(6).randn(n, 32).astype(np.float32)
    y = oracle.dense_spmm(ptr.numpy(), idx.numpy(), None, x, mean=True)
    deg = (ptr[1:] - ptr[:-1]).double()
    a = torch.sparse_csr_tensor(ptr.long(), idx.long(), torch.ones(idx.numel(), dtype=torch.float64),
                                size=(n, n))
    ref = (a @ torch.from_numpy(x).double()) / deg.clamp(min=1)[:, None]
    assert np.allclose(y, ref.numpy(), rtol=1e-5, atol=1e-5)


def test_warp4_chunk_rule():
    ptr = np.array([0, 0, 3, 3 + 130, 3 + 130 + 64], np.int32)
    t = oracle.warp4(ptr)
    assert t.tolist() == [[1, 0, 3, 0], [2, 3, 64, 0], [2, 67, 64, 0], [2, 131, 2, 0],
                          [3, 133, 64, 0]]


# ---------------------------------------------------------------- golden fixtures
def test_golden_inputs_regenerate(golden):
    ptr, idx = graphs.synthetic_csr(512, 16_000, seed=97)
    assert np.array_equal(golden["ptr"], ptr.numpy())
    assert np.array_equal(golden["idx"], idx.numpy())
    assert np.array_equal(golden["val"], graphs.sage_mean_values(ptr).numpy())


@pytest.mark.parametrize("k", [8, 16, 24, 32, 64])
def test_golden_oracle_topk(golden, k):
    d, i = oracle.maxk(golden["h"], k, "exact")
    assert np.array_equal(d, golden[f"exact_data_k{k}"])
    assert np.array_equal(i, golden[f"exact_index_k{k}"])
    d, i = oracle.maxk(golden["h"], k, "ref_compat")
    assert np.array_equal(d, golden[f"ref_data_k{k}"])
    assert np.array_equal(i, golden[f"ref_index_k{k}"])


@pytest.mark.parametrize("k", [8, 16, 24, 32, 64])
def test_golden_oracle_aggregation(golden, k):
    i = golden[f"exact_index_k{k}"]
    gs = oracle.sspmm_backward(golden["ptr"], golden["idx"], golden["val"], golden["g"], i)
    assert np.array_equal(gs, golden[f"bwd_k{k}"])
    if f"fwd_k{k}" in golden:
        y = oracle.spgemm_forward(golden["ptr"], golden["idx"], golden["val"],
                                  golden[f"exact_data_k{k}"], i, golden["h"].shape[1])
        assert np.array_equal(y, golden[f"fwd_k{k}"])
    assert np.array_equal(oracle.warp4(golden["ptr"]), golden["warp4"])
