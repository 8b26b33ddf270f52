"""Synthetic graph generators (CPU): the BASELINE generator and the locality-bearing
community variant used for the supplementary measurements."""
import torch

from maxk_kernels import graphs


def _rows(ptr):
    return torch.repeat_interleave(torch.arange(ptr.numel() - 1), (ptr[1:] - ptr[:-1]).long())


def _check_csr(ptr, idx, n):
    assert ptr.dtype == torch.int32 and idx.dtype == torch.int32
    assert int(ptr[0]) == 0 and int(ptr[-1]) == idx.numel()
    rows = _rows(ptr).long()
    key = rows * n + idx.long()
    assert torch.all(key[1:] > key[:-1])                  # sorted, no duplicate columns
    assert int((rows == idx.long()).sum()) == n           # one self-loop per row
    assert int(idx.min()) >= 0 and int(idx.max()) < n
    return rows


def test_synthetic_csr_exact_edge_count():
    ptr, idx = graphs.synthetic_csr(3000, 90_000, seed=5)
    _check_csr(ptr, idx, 3000)
    assert idx.numel() == 90_000


def test_community_csr_locality_and_shuffle():
    n, c = 6000, 12
    ptr, idx = graphs.community_csr(n, 200_000, communities=c, p_in=0.76, seed=3)
    rows = _check_csr(ptr, idx, n)
    size = -(-n // c)
    same = ((rows // size) == (idx.long() // size)).float().mean().item()
    # p_in inside the community plus the uniform draws that land there; duplicates merged
    assert 0.7 < same < 0.85
    assert 0.9 * 200_000 < idx.numel() <= 200_000
    sp, si = graphs.community_csr(n, 200_000, communities=c, p_in=0.76, seed=3, shuffle=True)
    srows = _check_csr(sp, si, n)
    assert si.numel() == idx.numel()                      # a relabelling keeps every edge
    same_s = ((srows // size) == (si.long() // size)).float().mean().item()
    assert same_s < 0.2                                   # structure hidden from ID order
    # same multiset of degrees
    assert torch.equal(torch.sort(ptr[1:] - ptr[:-1]).values, torch.sort(sp[1:] - sp[:-1]).values)


def test_community_csr_deterministic():
    a = graphs.community_csr(2000, 40_000, seed=9)
    b = graphs.community_csr(2000, 40_000, seed=9)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


def test_load_npz_csr_coo_and_csr(tmp_path):
    """scipy save_npz adjacency (the DGL dataset cache format) -> destination-row CSR with
    self-loops: row v lists the sources u of edges u -> v."""
    import numpy as np
    import scipy.sparse as sps
    rng = np.random.default_rng(4)
    n, m = 500, 4000
    src = rng.integers(0, n, m)
    dst = rng.integers(0, n, m)
    keep = src != dst
    src, dst = src[keep], dst[keep]
    key = np.unique(dst * n + src)
    dst, src = key // n, key % n
    coo = sps.coo_matrix((np.ones(src.size, np.float32), (src, dst)), shape=(n, n))
    ref = sps.csr_matrix((np.ones(src.size + n), (np.r_[dst, np.arange(n)], np.r_[src, np.arange(n)])),
                         shape=(n, n))
    ref.sort_indices()
    for i, mat in enumerate((coo, coo.tocsr(), coo.tocsc())):
        path = tmp_path / f"g{i}.npz"
        sps.save_npz(path, mat)
        ptr, idx = graphs.load_npz_csr(str(path))
        _check_csr(ptr, idx, n)
        assert np.array_equal(ptr.numpy(), ref.indptr)
        assert np.array_equal(idx.numpy(), ref.indices)
    assert graphs.find_dgl_graph("reddit", root=str(tmp_path)) is None
    (tmp_path / "reddit").mkdir()
    sps.save_npz(tmp_path / "reddit" / "reddit_graph.npz", coo)
    assert graphs.find_dgl_graph("reddit", root=str(tmp_path)).endswith("reddit_graph.npz")
