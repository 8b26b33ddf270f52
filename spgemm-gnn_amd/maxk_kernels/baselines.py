"""Comparators for the benchmarks (not on the MaxK path).

``spmm_rocsparse`` / ``spmm_rocsparse_coo`` are the MI355X counterparts of the reference's
cuSPARSE baselines ``spmm_cusparse`` (SO@0x243a0) and ``spmm_cusparse_coo`` (SO@0x24700;
SURVEY §2 L1, §8(a) a10): Y = A X with A CSR (or COO) int32/f32 and X row-major, through
rocSPARSE's generic SpMM (csrc/baseline_rocsparse.cpp, built into its own
libmaxk_baseline.so so the product library does not link rocSPARSE).
"""
from __future__ import annotations

import ctypes
import os
from typing import Tuple

import torch

_LIB = None
SPMM_ALGS = {"default": 0, "csr": 1, "csr_row_split": 4, "csr_merge": 5, "csr_merge_path": 9}
COO_ALGS = {"default": 0, "coo_segmented": 2, "coo_atomic": 3, "coo_segmented_atomic": 6}


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmaxk_baseline.so")
        lib = ctypes.CDLL(path)
        lib.maxk_spmm_rocsparse.restype = ctypes.c_int
        lib.maxk_spmm_rocsparse.argtypes = [ctypes.c_void_p] * 5 + [
            ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
            ctypes.POINTER(ctypes.c_float), ctypes.c_void_p]
        lib.maxk_spmm_rocsparse_coo.restype = ctypes.c_int
        lib.maxk_spmm_rocsparse_coo.argtypes = lib.maxk_spmm_rocsparse.argtypes
        lib.maxk_baseline_last_error.restype = ctypes.c_char_p
        _LIB = lib
    return _LIB


def _run(fn, a: torch.Tensor, idx: torch.Tensor, val: torch.Tensor, x: torch.Tensor,
         times: int, alg: int) -> Tuple[torch.Tensor, float]:
    n, d = x.shape
    y = torch.empty_like(x)
    ms = ctypes.c_float(0.0)
    vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    with torch.cuda.device(x.device):
        rc = fn(vp(a), vp(idx), vp(val), vp(x), vp(y), n, idx.numel(), d, alg, int(times),
                ctypes.byref(ms), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    if rc != 0:
        raise RuntimeError("maxk_kernels: " + _lib().maxk_baseline_last_error().decode())
    return y, float(ms.value)


def spmm_rocsparse(ptr: torch.Tensor, idx: torch.Tensor, val: torch.Tensor, x: torch.Tensor,
                   times: int = 0, alg: str = "default") -> Tuple[torch.Tensor, float]:
    """(Y = A @ X, mean ms of one timed rocsparse_spmm compute call; the warm-up's time when
    times == 0)."""
    return _run(_lib().maxk_spmm_rocsparse, ptr, idx, val, x, times, SPMM_ALGS[alg])


def coo_rows(ptr: torch.Tensor) -> torch.Tensor:
    """Row id of every edge of a CSR (int32 [E], ascending): the COO form's row array."""
    n = ptr.numel() - 1
    return torch.repeat_interleave(torch.arange(n, dtype=torch.int32, device=ptr.device),
                                   (ptr[1:] - ptr[:-1]).to(torch.int64)).contiguous()


def spmm_rocsparse_coo(rows: torch.Tensor, idx: torch.Tensor, val: torch.Tensor,
                       x: torch.Tensor, times: int = 0,
                       alg: str = "default") -> Tuple[torch.Tensor, float]:
    """``spmm_rocsparse`` with A in COO form (``rows`` from ``coo_rows(ptr)``)."""
    return _run(_lib().maxk_spmm_rocsparse_coo, rows, idx, val, x, times, COO_ALGS[alg])
