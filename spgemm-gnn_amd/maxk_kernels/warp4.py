"""Compatibility with the reference's ``.warp4`` partition metadata.

The reference reads ``../w12_nz64_warp_4/<name>.warp4`` (name hard-coded ``"graph"``)
on every SpGEMM call (SPMM_MAXK::do_test SO@0x24bf0, cuda_read_array<int> SO@0x252c0);
the writer ``generate_meta.py`` is absent (README.md:86). Format: raw
little-endian int32 quads ``{row, first_nz, len, 0}``, each CSR row cut into consecutive
chunks of <= 64 nonzeros, no header. The gfx950 kernels do not need it (they partition
from ``ptr`` on the device); these helpers let reference-generated metadata be checked
against a graph, and produce it for tools that expect it.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from ._lib import check, lib

WARP_MAX_NZ = 64
DEFAULT_DIR = os.path.join("..", "w12_nz64_warp_4")


def build_warp4(ptr, max_nz: int = WARP_MAX_NZ) -> np.ndarray:
    """[W, 4] int32 chunk table for the CSR row pointer ``ptr`` (any array-like)."""
    hp = np.ascontiguousarray(np.asarray(ptr.cpu() if hasattr(ptr, "cpu") else ptr),
                              dtype=np.int32)
    n = hp.size - 1
    count = ctypes.c_int64(0)
    check(lib.maxk_warp4_build(hp.ctypes.data, n, max_nz, None, 0, ctypes.byref(count)),
          "maxk_warp4_build")
    out = np.zeros((count.value, 4), dtype=np.int32)
    if count.value:
        check(lib.maxk_warp4_build(hp.ctypes.data, n, max_nz, out.ctypes.data, count.value,
                                   ctypes.byref(count)), "maxk_warp4_build")
    return out


def write_warp4(path: str, table: np.ndarray) -> None:
    np.ascontiguousarray(table, dtype="<i4").tofile(path)


def read_warp4(path: str) -> np.ndarray:
    raw = np.fromfile(path, dtype="<i4")
    if raw.size % 4:
        raise ValueError(f"{path}: size {raw.size * 4} B is not a multiple of 16")
    return raw.reshape(-1, 4)


def warp4_path(name: str = "graph", directory: str = DEFAULT_DIR) -> str:
    """Path the reference would open: ``../w12_nz64_warp_4/<name>.warp4``."""
    return os.path.join(directory, f"{name}.warp4")


def _as_table(table) -> np.ndarray:
    t = np.asarray(table)
    if t.ndim != 2 or t.shape[1] != 4:
        raise ValueError(f"warp4 table must be [W, 4], got shape {t.shape}")
    return t.astype(np.int64, copy=False)


def ptr_from_warp4(table, num_nodes: int, max_nz: int = WARP_MAX_NZ) -> np.ndarray:
    """Rebuild the CSR row pointer a ``.warp4`` chunk table describes.

    The reference kernels only ever see the chunks (``SPMM_MAXK::do_test`` SO@0x24bf0 hands
    ``warp4`` to ``spmm_kernel_opt2_sparse_v3``; ``ptr`` at object +0x10 is unused, SURVEY
    §8 a4), so a replayed file defines the partition by itself. Every row's chunks must tile
    one consecutive nonzero range, the ranges must follow row order from 0 without gaps, each
    chunk holds 1..``max_nz`` nonzeros and its 4th word is 0 (the k < 32 fallback reads it as a
    length). Rows without chunks get degree 0. Raises ValueError otherwise."""
    t = _as_table(table)
    if num_nodes < 0:
        raise ValueError("num_nodes must be >= 0")
    if t.shape[0] == 0:
        return np.zeros(num_nodes + 1, np.int32)
    row, first, length, pad = t[:, 0], t[:, 1], t[:, 2], t[:, 3]
    if np.any(pad != 0):
        raise ValueError(f"warp4 chunk {int(np.flatnonzero(pad != 0)[0])}: 4th word must be 0")
    if np.any((row < 0) | (row >= num_nodes)):
        raise ValueError(f"warp4 chunk {int(np.flatnonzero((row < 0) | (row >= num_nodes))[0])}:"
                         f" row out of range [0, {num_nodes})")
    if np.any((length < 1) | (length > max_nz)):
        bad = int(np.flatnonzero((length < 1) | (length > max_nz))[0])
        raise ValueError(f"warp4 chunk {bad}: length {int(length[bad])} not in [1, {max_nz}]")
    order = np.lexsort((first, row))
    r, f, ln = row[order], first[order], length[order]
    # Sorted by (row, first_nz), consecutive chunks must abut: the whole table tiles [0, E).
    ends = f + ln
    if f[0] != 0:
        raise ValueError(f"warp4: the first chunk starts at nonzero {int(f[0])}, not 0")
    gap = np.flatnonzero(f[1:] != ends[:-1])
    if gap.size:
        i = int(gap[0]) + 1
        raise ValueError(f"warp4: chunk (row {int(r[i])}, first_nz {int(f[i])}) does not follow "
                         f"the previous chunk's end {int(ends[i - 1])} (gap or overlap)")
    if int(ends[-1]) >= 2 ** 31:
        raise ValueError("warp4: more than 2^31 - 1 nonzeros")
    deg = np.bincount(r, weights=ln, minlength=num_nodes).astype(np.int64)
    ptr = np.zeros(num_nodes + 1, np.int64)
    np.cumsum(deg, out=ptr[1:])
    return ptr.astype(np.int32)


def validate_warp4(table, ptr, max_nz: int = WARP_MAX_NZ, strict: bool = False) -> None:
    """Check a (reference-generated) ``.warp4`` table against the graph's CSR ``ptr``.

    Non-strict: the chunks describe exactly ``ptr``'s rows (see ``ptr_from_warp4``), so the
    reference kernels would sum the same nonzeros as the plan built from ``ptr``. Strict: the
    table is also the canonical chunking of ``generate_meta.py`` (consecutive chunks of
    ``max_nz`` in CSR order, README_INTEGRATED.md:252-262), entry for entry."""
    hp = np.asarray(ptr.cpu() if hasattr(ptr, "cpu") else ptr).astype(np.int64)
    n = hp.size - 1
    got = ptr_from_warp4(table, n, max_nz).astype(np.int64)
    if not np.array_equal(got, hp):
        bad = int(np.flatnonzero(got != hp)[0])
        raise ValueError(f"warp4 does not match ptr: row pointer {bad} is {int(got[bad])} "
                         f"in the table, {int(hp[bad])} in the graph")
    if strict and not np.array_equal(_as_table(table), build_warp4(hp, max_nz).astype(np.int64)):
        raise ValueError("warp4 matches ptr but is not the canonical chunking")


def replay_warp4(ptr, name: str = "graph", directory: str = DEFAULT_DIR,
                 max_nz: int = WARP_MAX_NZ, strict: bool = False) -> np.ndarray:
    """Read the file the reference would open for ``name`` and validate it against ``ptr``.

    Returns the table. The gfx950 plan is still built from ``ptr`` on the device (the chunk
    table is never uploaded); a table that passes describes the same nonzero sums."""
    table = read_warp4(warp4_path(name, directory))
    validate_warp4(table, ptr, max_nz, strict)
    return table
