"""ctypes binding of the C ABI in include/maxk_hip.h (libmaxk_hip.so, built in-tree).

The library is the product: there is no Python or CPU fallback. If the shared object is
missing or cannot be loaded, importing :mod:`maxk_kernels` raises ImportError, exactly as
the reference's ``import maxk_kernels`` does when its extension is absent
(utils/maxk_layers.py:9-14).
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  -- must load torch's libamdhip64 before ours (same soname)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MAXK_HIP_LIB", os.path.join(_HERE, "libmaxk_hip.so"))

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64

# name -> (restype, argtypes); must match include/maxk_hip.h exactly.
SIGNATURES = {
    "maxk_abi_version": (ctypes.c_int, []),
    "maxk_last_error": (ctypes.c_char_p, []),
    "maxk_topk_cbsr": (ctypes.c_int, [_vp, _vp, _vp, _i32, _i32, _i32, _i32, _vp]),
    "maxk_topk_cbsr_count": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i32, _i32, _i32, _i32, _vp]),
    "maxk_topk_cbsr_tables": (ctypes.c_int, [_vp, _vp, _i64, _vp, _i64, _vp, _i32, _i32, _i32,
                                             _i32, _vp]),
    "maxk_topk_cbsr_ex": (ctypes.c_int, [_vp, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _i64, _i32,
                                         _i32, _i32, _i32, _vp]),
    "maxk_topk_stats_scratch_bytes": (ctypes.c_int64, [_i32]),
    "maxk_scatter_backward": (ctypes.c_int, [_vp, _vp, _vp, _i32, _i32, _i32, _vp]),
    "maxk_scatter_backward_tables": (ctypes.c_int, [_vp, _vp, _i64, _vp, _i32, _i32, _i32, _vp]),
    "maxk_plan_create": (ctypes.c_int, [_vp, _vp, _vp, _i32, _i64, _i32, _i32, _vp,
                                        ctypes.POINTER(_vp)]),
    "maxk_plan_create_rect": (ctypes.c_int, [_vp, _vp, _vp, _i32, _i32, _i64, _i32, _i32,
                                             _vp, ctypes.POINTER(_vp)]),
    "maxk_plan_create_ex": (ctypes.c_int, [_vp, _vp, _vp, _i32, _i32, _i64, _i32, _i32, _vp,
                                           _vp, ctypes.POINTER(_vp)]),
    "maxk_plan_create_sized": (ctypes.c_int, [_vp, _vp, _vp, _i32, _i32, _i64, _i32, _i32,
                                              _vp, _i64, _vp, _vp, ctypes.POINTER(_vp)]),
    "maxk_plan_refresh_values": (ctypes.c_int, [_vp, _vp, _vp]),
    "maxk_plan_get_info": (ctypes.c_int, [_vp, _vp]),
    "maxk_plan_get_info_sized": (ctypes.c_int, [_vp, _vp, _i64]),
    "maxk_plan_get_col_order": (ctypes.c_int, [_vp, _vp, _vp]),
    "maxk_cbsr_stats": (ctypes.c_int, [_vp, _vp, _i32, _i32, _vp, _vp]),
    "maxk_cbsr_stats_tables": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i32, _i32, _vp, _vp]),
    "maxk_spgemm_forward_tables": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _i64, _vp, _i64, _vp,
                                                  _i32, _i64, _i32, _i32, _i32, _vp, _i32, _i64,
                                                  _vp, _i64, _vp]),
    "maxk_sspmm_backward_tables": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _i32,
                                                  _i64, _i32, _i32, _vp, _i64, _vp]),
    "maxk_spgemm_forward_ex": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i64,
                                              _i32, _i32, _i32, _vp, _i32, _i64, _vp, _i64,
                                              _vp]),
    "maxk_plan_destroy": (ctypes.c_int, [_vp]),
    "maxk_spgemm_forward": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i64,
                                           _i32, _i32, _vp]),
    "maxk_spgemm_forward_acc": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i64,
                                               _i32, _i32, _vp]),
    "maxk_sspmm_backward": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i64,
                                           _i32, _i32, _vp]),
    "maxk_spgemm_forward_ws": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i64,
                                              _i32, _i32, _i32, _vp, _i64, _vp]),
    "maxk_sspmm_backward_ws": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i64,
                                              _i32, _i32, _vp, _i64, _vp]),
    "maxk_plan_workspace_bytes": (ctypes.c_int, [_vp, ctypes.POINTER(_i64),
                                                 ctypes.POINTER(_i64)]),
    "maxk_dense_spmm_csr": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _i32, _i32, _vp]),
    "maxk_warp4_build": (ctypes.c_int, [_vp, _i32, _i32, _vp, _i64, ctypes.POINTER(_i64)]),
}


class PlanOptions(ctypes.Structure):
    """Mirror of ``maxk_plan_options`` (0 = default for every field; the fields the header
    marks "ABI 3" accept only 0 or the behaviour that remains)."""

    _fields_ = [
        ("fwd_tile_rows", _i32),
        ("fwd_accumulator", _i32),
        ("bwd_lds_bytes", _i32),
        ("bwd_accumulator", _i32),
        ("bwd_tasks_per_cu", _i32),
        ("fwd_task_cap", _i32),
        ("bwd_features_per_lane", _i32),
        ("fwd_phases", _i32),
        ("fwd_persistent", _i32),
        ("fwd_unroll", _i32),
        ("bwd_unroll", _i32),
        ("bwd_order", _i32),
        ("bwd_slot_groups", _i32),
        ("bwd_min_task_edges", _i32),
        ("bwd_acc_pad", _i32),
        ("bwd_sel_lds", _i32),
        ("fwd_rotate", _i32),
        ("bwd_algo", _i32),
        ("fwd_waves", _i32),
        ("bwd_waves", _i32),
        ("fwd_prefetch", _i32),
        ("bwd_prefetch", _i32),
        ("fwd_record_bytes", _i32),
        ("fwd_branchless", _i32),
        ("fwd_chunk3", _i32),
        ("bwd_cas64", _i32),
        ("quad_loads", _i32),
        ("fwd_two_tables", _i32),
        ("fwd_rot_windows", _i32),
        ("fwd_rot_rate", _i32),
        ("external_workspace", _i32),
        ("bwd_flush", _i32),
        ("bwd_piece_edges", _i32),
        ("bwd_chunk_bounds", _i32),
        ("fwd_fixed", _i32),
        ("bwd_tp_store", _i32),
        # ABI 2 (maxk_plan_create_sized)
        ("bwd_row_cost", _i32),
        ("col_order", _i32),
        ("bwd_tp_chunks", _i32),
        ("bwd_row_order", _i32),
        # round 5
        ("fwd_handout", _i32),
        ("bwd_handout", _i32),
    ]


ACC_KINDS = {"auto": 0, "f64": 1, "f32_cas": 2}
# maxk_plan_options.col_order by name (MAXK_COL_ORDER_*; 3, clustered, was removed in ABI 3)
COL_ORDERS = {"auto": 0, "identity": 1, "scattered": 2, "given": 4}
# maxk_plan_options.bwd_algo / maxk_plan_info.bwd_algo (MAXK_BWD_*)
BWD_ALGOS = {"auto": 0, "column_blocks": 1, "two_pass": 3}


class PlanInfo(ctypes.Structure):
    """Mirror of ``maxk_plan_info``."""

    _fields_ = [
        ("num_nodes", _i32),
        ("num_edges", _i64),
        ("dim_origin", _i32),
        ("dim_k", _i32),
        ("fwd_tasks", _i32),
        ("fwd_split_rows", _i32),
        ("bwd_block_cols", _i32),
        ("bwd_blocks", _i32),
        ("bwd_tasks", _i32),
        ("bwd_shared_blocks", _i32),
        ("device_bytes", _i64),
        ("num_cols", _i32),
        ("bwd_algo", _i32),
        # ABI 2 (maxk_plan_get_info_sized)
        ("col_order", _i32),
        ("bwd_chunk_bounds", _i32),
        ("bwd_tp_chunks", _i32),
        ("bwd_row_order", _i32),
        ("bwd_workspace_peak", _i64),
        # round 5
        ("fwd_handout", _i32),
        ("bwd_handout", _i32),
        ("fwd_waves", _i32),
        ("fwd_unroll", _i32),
        ("bwd_waves", _i32),
        ("bwd_unroll", _i32),
        # ABI 4
        ("fwd_layout", _i32),
        ("fwd_record_bytes", _i32),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"maxk_kernels: native library {LIB_PATH} is missing; build it with "
            "`make -C spgemm-gnn_amd` (or __graft_entry__.build())")
    try:
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_LOCAL)
    except OSError as exc:  # pragma: no cover - depends on the box
        raise ImportError(f"maxk_kernels: cannot load {LIB_PATH}: {exc}") from exc
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def lib_sha256(path: str = LIB_PATH) -> str:
    """sha256 of the loaded libmaxk_hip.so: ties a measurement (profiles/pmc_traffic.json)
    to the kernel binary it was taken on."""
    import hashlib
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


class MaxKError(RuntimeError):
    """Raised for a non-zero return of the C ABI."""


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib.maxk_last_error()
        msg = msg.decode() if msg else ""
        raise MaxKError(f"maxk_kernels: {what} failed (code {rc}): {msg}")
