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
