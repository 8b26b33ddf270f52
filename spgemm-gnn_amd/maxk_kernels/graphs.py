"""Synthetic graphs with the benchmark datasets' (N, E) — no datasets are available offline.

Generator: per-row in-degrees from a seeded lognormal
(sigma 1.2; the reference publishes no degree histogram) scaled so that sum(deg) = E - N,
columns drawn uniformly without replacement (excluding the row itself) and sorted, plus
one self-loop per row (DGL ``AddSelfLoop``: run/reddit.log:28 reports 114,848,857 edges
after it). Seed 97 is the reference default (utils/config.py:54).

:func:`synthetic_csr` draws the columns from torch's generator (the tests' graphs);
:func:`synthetic_ptr` + :func:`synthetic_rows` (the bench graph since round 4) draw them from a
counter-based stream, so each rank of a row partition generates only its own rows.
"""
from __future__ import annotations

from typing import Optional

import torch

DATASETS = {
    # name: (num_nodes, num_edges incl. self-loops)   sources: SURVEY §6 / spgemm_plot.py
    "reddit": (232_965, 114_848_857),
    "ogbn-products": (2_449_029, 123_718_280),
    "ogbn-proteins": (132_534, 79_122_504),
    "flickr": (89_250, 989_006 + 89_250),
    "yelp": (716_847, 13_954_819 + 716_847),
}


def lognormal_degrees(n: int, total: int, sigma: float, gen: torch.Generator,
                      device) -> torch.Tensor:
    """int64 [n] degrees in [0, n-1] summing exactly to ``total``."""
    if n <= 1:
        return torch.zeros(n, dtype=torch.int64, device=device)
    total = min(total, n * (n - 1))
    z = torch.randn(n, generator=gen, device=device, dtype=torch.float64)
    w = torch.exp(sigma * z)
    exact = w / w.sum() * total
    deg = torch.floor(exact).clamp_(max=n - 1).to(torch.int64)
    rem = int(total - int(deg.sum()))
    while rem > 0:
        room = deg < (n - 1)
        frac = torch.where(room, exact - deg.to(torch.float64), torch.full_like(exact, -1.0))
        take = min(rem, int(room.sum()))
        top = torch.topk(frac, take).indices
        deg[top] += 1
        rem -= take
    return deg


def synthetic_csr(num_nodes: int, num_edges: int, seed: int = 97, sigma: float = 1.2,
                  device="cpu", self_loops: bool = True):
    """Destination-row CSR (ptr int32 [N+1], idx int32 [E]) with sorted columns."""
    device = torch.device(device)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    n = int(num_nodes)
    extra = n if self_loops else 0
    deg = lognormal_degrees(n, int(num_edges) - extra, sigma, gen, device)
    m = int(deg.sum())
    rows = torch.repeat_interleave(torch.arange(n, device=device), deg)
    # s ~ U{0 .. n-2-deg}: a sorted multiset of deg draws; t_i = s_i + i is then a sorted
    # deg-subset of [0, n-1); shifting t >= row by one excludes the row itself.
    span = (n - 1 - deg)[rows] + 1
    s = torch.floor(torch.rand(m, generator=gen, device=device, dtype=torch.float64)
                    * span.to(torch.float64)).to(torch.int64)
    s = torch.minimum(s, span - 1)
    key = rows * n + s
    key, _ = torch.sort(key)
    s = key - rows * n
    start = torch.cumsum(deg, 0) - deg
    local = torch.arange(m, device=device) - start[rows]
    cols = s + local
    cols = cols + (cols >= rows).to(torch.int64)
    del key, s, local, span
    if self_loops:
        ar = torch.arange(n, device=device)
        rows = torch.cat([rows, ar])
        cols = torch.cat([cols, ar])
        key, _ = torch.sort(rows * n + cols)
        rows = key // n
        cols = key - rows * n
        deg = deg + 1
        del key
    ptr = torch.zeros(n + 1, dtype=torch.int64, device=device)
    ptr[1:] = torch.cumsum(deg, 0)
    return ptr.to(torch.int32), cols.to(torch.int32)


_M64 = (1 << 64) - 1


def _i64(c: int) -> int:
    """A 64-bit constant as the int64 value with the same bits (torch has no uint64 math)."""
    return c - (1 << 64) if c >= (1 << 63) else c


def _srl(z: torch.Tensor, s: int) -> torch.Tensor:
    """Logical right shift of int64 bit patterns."""
    return (z >> s) & ((1 << (64 - s)) - 1)


def hash_uniform(seed: int, index: torch.Tensor) -> torch.Tensor:
    """Counter-based uniforms: splitmix64(seed * 2^32 + index) -> float64 in [0, 1) (53 bits).
    Element i depends only on (seed, index[i]), so any slice of a stream (one rank's edges)
    can be generated alone and equals that slice of the whole stream. int64 products wrap
    modulo 2^64 as the unsigned arithmetic of splitmix64 does."""
    z = index.to(torch.int64) + (int(seed) << 32) + _i64(0x9E3779B97F4A7C15)
    z = (z ^ _srl(z, 30)) * _i64(0xBF58476D1CE4E5B9)
    z = (z ^ _srl(z, 27)) * _i64(0x94D049BB133111EB)
    z = z ^ _srl(z, 31)
    return _srl(z, 11).to(torch.float64) * (2.0 ** -53)


def synthetic_ptr(num_nodes: int, num_edges: int, seed: int = 97, sigma: float = 1.2,
                  device="cpu") -> torch.Tensor:
    """ptr (int32 [N+1]) of :func:`synthetic_rows`'s graph: lognormal degrees (the same
    generator as :func:`synthetic_csr`) plus one self-loop per row. O(N): every rank of a
    row partition computes it to balance its rows before generating only those."""
    device = torch.device(device)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    n = int(num_nodes)
    deg = lognormal_degrees(n, int(num_edges) - n, sigma, gen, device) + 1
    ptr = torch.zeros(n + 1, dtype=torch.int64, device=device)
    ptr[1:] = torch.cumsum(deg, 0)
    return ptr.to(torch.int32)


def synthetic_rows(ptr: torch.Tensor, seed: int = 97, rows=None) -> torch.Tensor:
    """Column ids (int32, sorted per row) of rows [r0, r1) of the graph whose ptr is
    :func:`synthetic_ptr`'s: row r holds its self-loop plus deg(r) - 1 columns drawn uniformly
    without replacement from the other nodes, the draws of its edges coming from the
    counter-based stream :func:`hash_uniform` at the edges' global positions. A rank that
    generates only its rows gets exactly those rows of the whole graph (bench.py: every
    world size benchmarks the same graph, and no rank builds the 115 M-edge whole).
    Host syncs: one (the two edge offsets)."""
    n = ptr.numel() - 1
    r0, r1 = (0, n) if rows is None else (int(rows[0]), int(rows[1]))
    dev = ptr.device
    p = ptr[r0:r1 + 1].to(torch.int64)
    e0, e1 = (int(x) for x in torch.stack([p[0], p[-1]]).tolist())
    deg = p[1:] - p[:-1] - 1                          # draws per row (self-loop excluded)
    m = e1 - e0 - (r1 - r0)
    rl = torch.repeat_interleave(torch.arange(r1 - r0, device=dev), deg, output_size=m)
    row = rl + r0
    # draw j of row r: uniform index in [0, n - 1 - deg(r)]; sorted, t_j = s_j + j is a sorted
    # deg-subset of [0, n - 1); shifting t >= r by one excludes the row itself
    start = torch.cumsum(deg, 0) - deg
    gpos = (p[:-1] - (torch.arange(r1 - r0, device=dev) + r0))[rl] + (torch.arange(m, device=dev) - start[rl])
    span = (n - 1 - deg)[rl] + 1
    s = torch.floor(hash_uniform(seed, gpos) * span.to(torch.float64)).to(torch.int64)
    s = torch.minimum(s, span - 1)
    key, _ = torch.sort(rl * n + s)
    s = key - rl * n
    cols = s + (torch.arange(m, device=dev) - start[rl])
    cols = cols + (cols >= row).to(torch.int64)
    del key, s, span, gpos
    ar = torch.arange(r1 - r0, device=dev)
    key, _ = torch.sort(torch.cat([rl, ar]) * n + torch.cat([cols, ar + r0]))
    return (key - (key // n) * n).to(torch.int32)


def community_csr(num_nodes: int, num_edges: int, communities: int = 41, p_in: float = 0.76,
                  seed: int = 97, sigma: float = 1.2, shuffle: bool = False, device="cpu"):
    """A locality-bearing variant of :func:`synthetic_csr` (supplementary measurements only,
    DESIGN §6): the same lognormal row degrees, but each edge's column is drawn, with
    probability ``p_in``, uniformly inside the row's community and otherwise uniformly over
    all nodes. Communities are contiguous ID blocks of ~N/communities nodes. The defaults
    follow the Reddit dataset: 41 subreddit classes and an edge homophily of about 0.76.
    Duplicate columns are merged, so E comes out slightly below ``num_edges``; one self-loop
    per row. ``shuffle``: relabel the nodes by a seeded random permutation. That keeps the
    community structure but hides it from ID order, as a dataset's arbitrary node ids do.
    Returns (ptr int32 [N+1], idx int32 [E]) with sorted columns."""
    device = torch.device(device)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    n = int(num_nodes)
    c = max(1, min(int(communities), n))
    deg = lognormal_degrees(n, int(num_edges) - n, sigma, gen, device)
    m = int(deg.sum())
    rows = torch.repeat_interleave(torch.arange(n, device=device), deg)
    size = -(-n // c)
    lo = (rows // size) * size
    width = torch.clamp(n - lo, max=size)
    u = torch.rand(m, generator=gen, device=device, dtype=torch.float64)
    inside = torch.rand(m, generator=gen, device=device) < p_in
    cols = torch.where(inside, lo + (u * width.to(torch.float64)).to(torch.int64),
                       (u * n).to(torch.int64))
    cols = torch.minimum(cols, torch.full_like(cols, n - 1))
    ar = torch.arange(n, device=device)
    rows = torch.cat([rows, ar])
    cols = torch.cat([cols, ar])
    if shuffle:
        perm = torch.randperm(n, generator=gen, device=device)
        rows, cols = perm[rows], perm[cols]
    key = torch.unique(rows * n + cols)  # sorted, duplicates merged
    rows = key // n
    cols = key - rows * n
    ptr = torch.zeros(n + 1, dtype=torch.int64, device=device)
    ptr[1:] = torch.cumsum(torch.bincount(rows, minlength=n), 0)
    return ptr.to(torch.int32), cols.to(torch.int32)


def row_degrees(ptr: torch.Tensor) -> torch.Tensor:
    return (ptr[1:] - ptr[:-1]).to(torch.int64)


def sage_mean_values(ptr: torch.Tensor, num_edges: Optional[int] = None) -> torch.Tensor:
    """val[nz] = 1/deg(row) (SAGE mean; utils/maxk_layers.py:147-157). ``num_edges``
    (= ptr[-1] - ptr[0], when the caller knows it) spares the host sync that
    ``repeat_interleave`` otherwise makes to size its output."""
    deg = row_degrees(ptr)
    inv = 1.0 / deg.clamp(min=1).to(torch.float32)
    return torch.repeat_interleave(inv, deg, output_size=num_edges)


def gcn_values(ptr: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """val[nz] = deg(r)^-1/2 * deg(c)^-1/2 (symmetric GCN normalisation with in-degrees;
    utils/maxk_layers.py:314-317,373-376)."""
    deg = row_degrees(ptr).clamp(min=1).to(torch.float32)
    nr = deg.rsqrt()
    rows = torch.repeat_interleave(torch.arange(deg.numel(), device=ptr.device),
                                   row_degrees(ptr))
    return nr[rows] * nr[idx.to(torch.int64)]


def features(num_nodes: int, dim: int, seed: int, device="cpu",
             gen_device: Optional[str] = None) -> torch.Tensor:
    """N(0, 1) f32 [num_nodes, dim] from a seeded generator."""
    gd = torch.device(gen_device or device)
    g = torch.Generator(device=gd)
    g.manual_seed(seed)
    return torch.randn(num_nodes, dim, generator=g, device=gd).to(device)


# DGL's on-disk dataset cache (``dgl.data.RedditDataset`` et al.): <root>/<dir>/<file>. The
# graph file is a scipy.sparse ``save_npz`` archive of the symmetric adjacency, without
# self-loops. Used by bench.py when it exists on the box.
DGL_GRAPH_FILES = {"reddit": ("reddit", "reddit_graph.npz")}


def find_dgl_graph(name: str, root: Optional[str] = None) -> Optional[str]:
    """Path of the DGL cache file for dataset ``name`` if it exists, else None."""
    import os
    if name not in DGL_GRAPH_FILES:
        return None
    root = root or os.environ.get("DGL_DOWNLOAD_DIR") or os.path.expanduser("~/.dgl")
    sub, fname = DGL_GRAPH_FILES[name]
    path = os.path.join(root, sub, fname)
    return path if os.path.isfile(path) else None


def load_npz_csr(path: str, self_loops: bool = True, device="cpu"):
    """Destination-row CSR (ptr int32 [N+1], idx int32 [E], sorted columns) from a
    scipy.sparse ``save_npz`` archive (COO or CSR/CSC). Read with ``numpy.load`` and
    ``allow_pickle=False``: nothing in the file is executed. Edge (u, v) of the archive is
    DGL's edge u -> v, so destination row v lists its sources u (DGL's in-edge CSR,
    ``adj_tensors('csc')``). ``self_loops`` appends one (v, v) per node, as DGL's
    ``AddSelfLoop`` does (run/reddit.log:28 counts 114,848,857 edges after it)."""
    import numpy as np
    with np.load(path, allow_pickle=False) as z:
        fmt = z["format"].item()
        fmt = fmt.decode() if isinstance(fmt, bytes) else str(fmt)
        shape = tuple(int(x) for x in z["shape"])
        if fmt == "coo":
            src, dst = z["row"].astype(np.int64), z["col"].astype(np.int64)
        elif fmt in ("csr", "csc"):
            indptr, indices = z["indptr"].astype(np.int64), z["indices"].astype(np.int64)
            major = np.repeat(np.arange(indptr.size - 1, dtype=np.int64), np.diff(indptr))
            src, dst = (major, indices) if fmt == "csr" else (indices, major)
        else:
            raise ValueError(f"{path}: unsupported sparse format {fmt!r}")
    if shape[0] != shape[1]:
        raise ValueError(f"{path}: adjacency must be square, got {shape}")
    n = shape[0]
    rows = torch.from_numpy(dst).to(device)
    cols = torch.from_numpy(src).to(device)
    if self_loops:
        ar = torch.arange(n, device=rows.device)
        rows, cols = torch.cat([rows, ar]), torch.cat([cols, ar])
    key, _ = torch.sort(rows * n + cols)
    rows = key // n
    cols = key - rows * n
    ptr = torch.zeros(n + 1, dtype=torch.int64, device=rows.device)
    ptr[1:] = torch.cumsum(torch.bincount(rows, minlength=n), 0)
    return ptr.to(torch.int32), cols.to(torch.int32)


def bench_csr(name: str, device="cpu", seed: int = 97):
    """(ptr, idx) of the bench graph shaped like dataset ``name``: :func:`synthetic_ptr` +
    :func:`synthetic_rows` (bench.py's graph at every world size; the tools time this one)."""
    n, e = DATASETS[name]
    ptr = synthetic_ptr(n, e, seed=seed, device=device)
    return ptr, synthetic_rows(ptr, seed=seed)


def dataset_csr(name: str, device="cpu", seed: int = 97):
    return bench_csr(name, device=device, seed=seed)
