"""The four functions of the reference's ``maxk_kernels`` extension, on the gfx950 C ABI.

Reference binding: pybind11 module ``maxk_kernels`` (PyInit SO@0xfc90) with the wrappers
``maxk_forward`` (SO@0xe340), ``maxk_backward`` (SO@0xe690), ``spgemm_forward``
(SO@0xea20) and ``spgemm_backward`` (SO@0xf170); argument checks recovered from
``kernels/maxk_bindings.cpp`` lines 27-30, 34-36, 45-54, 65-71.

Same names, same positional signatures, same return shapes and the same RuntimeError
messages for the same checks. Differences (all fixes of SURVEY §8(b) defects):

* kernels are launched on the current HIP stream with no device-wide synchronisation;
* ``spgemm_forward/backward`` derive their partition metadata from ``ptr`` (cached per
  graph) instead of reading ``../w12_nz64_warp_4/graph.warp4`` and printing to stdout;
* ``maxk_backward`` returns a stable ``[N, D]`` shape when ``dim_origin`` is given;
* ``maxk_forward`` can also return ``sp_index`` (the reference computes and drops it).
"""
from __future__ import annotations

import collections
import contextlib
import ctypes
import os
import threading
from typing import Optional, Tuple

import torch

from ._lib import ACC_KINDS, BWD_ALGOS, COL_ORDERS, PlanInfo, PlanOptions, check, lib

TOPK_MODES = {"exact": 0, "ref_compat": 1}


def _stream() -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t: Optional[torch.Tensor]) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr() if t is not None else 0)


_SAME_DEVICE = contextlib.nullcontext()


def _device(dev: torch.device):
    """``torch.cuda.device(dev)``, or a no-op when ``dev`` is already current (host cost)."""
    return _SAME_DEVICE if dev.index == torch.cuda.current_device() else torch.cuda.device(dev)


def _need(cond: bool, msg: str) -> None:
    if not cond:
        raise RuntimeError(msg)


def _check_tensor(t: torch.Tensor, name: str, dtype: Optional[torch.dtype] = None) -> None:
    _need(isinstance(t, torch.Tensor), f"{name} must be a tensor")
    _need(t.is_cuda, f"{name} must be a CUDA tensor")
    _need(t.is_contiguous(), f"{name} must be contiguous")
    if dtype is not None:
        _need(t.dtype == dtype, f"{name} must be {str(dtype).replace('torch.', '')}")


def _table(t: torch.Tensor, name: str, dtype: torch.dtype, rows: int, k: int) -> int:
    """A [rows, k] CBSR table whose rows may be strided (interleaved records): returns the row
    stride in elements."""
    _need(isinstance(t, torch.Tensor) and t.is_cuda, f"{name} must be a CUDA tensor")
    _need(t.dtype == dtype, f"{name} must be {str(dtype).replace('torch.', '')}")
    _need(t.dim() == 2 and tuple(t.shape) == (rows, k), f"{name} must be [{rows}, {k}]")
    _need(t.stride(1) == 1 and (rows <= 1 or t.stride(0) >= k),
          f"{name} must have unit column stride and row stride >= k")
    return t.stride(0) if rows > 1 else k


# -------------------------------------------------------------------------------------
# MaxK top-k
# -------------------------------------------------------------------------------------
def maxk_forward(input: torch.Tensor, k: int, mode: str = "exact",
                 return_index: bool = False, out=None, return_count: bool = False,
                 stats: Optional[torch.Tensor] = None):
    """MaxK nonlinearity -> CBSR. Reference: ``maxk_forward(input, k) -> [N, k] f32``.

    Checks (bindings.cpp:27-30): "input must be a CUDA tensor", "input must be
    contiguous", "Input must be 2D tensor", "k must be between 1 and input dimension".
    ``mode='exact'`` selects the true top-k (utils/models.py:14 semantics), ``'ref_compat'``
    the reference kernel's 8-step bisection, bit-exact. With ``return_index=True`` returns
    ``(sp_data, sp_index)`` with ``sp_index`` u8 ``[N, k]`` in ascending feature order.
    ``out=(sp_data, sp_index)`` writes into caller-owned ``[N, k]`` tables with unit column
    stride (rows may be strided: the interleaved send records of
    :class:`maxk_kernels.dist.ShardedAggregation`). ``return_count=True``
    appends the int32 ``[N]`` number of filled slots per row (``k`` in exact mode; in
    ref_compat mode the slots past it are the reference's ``(0.0f, 0)`` padding).
    ``stats``: a contiguous int32 CUDA tensor of 2 elements (e.g. a view into a record) that
    receives the fixed-point statistics of the emitted table with the top-k
    (``maxk_topk_cbsr_ex``; its scratch comes from torch's caching allocator): the pair
    :meth:`GraphPlan.forward` takes as ``stats=stats.view(1, 2)`` instead of its own pass over
    the table.
    """
    _need(input.is_cuda, "input must be a CUDA tensor")
    _need(input.is_contiguous(), "input must be contiguous")
    _need(input.dim() == 2, "Input must be 2D tensor")
    n, d = input.shape
    _need(1 <= k <= d, "k must be between 1 and input dimension")
    _need(d <= 256, "input dimension must be <= 256 (u8 selectors)")
    _need(input.dtype == torch.float32, "input must be float32")
    _need(mode in TOPK_MODES, f"mode must be one of {sorted(TOPK_MODES)}")
    if out is None:
        sp_data = torch.empty((n, k), dtype=torch.float32, device=input.device)
        sp_index = torch.empty((n, k), dtype=torch.uint8, device=input.device)
        ds = is_ = k
    else:
        sp_data, sp_index = out
        _need(sp_data.device == input.device and sp_index.device == input.device,
              "out must be on the input's device")
        ds = _table(sp_data, "out[0]", torch.float32, n, k)
        is_ = _table(sp_index, "out[1]", torch.uint8, n, k)
    count = torch.empty(n, dtype=torch.int32, device=input.device) if return_count else None
    scratch, sbytes = None, 0
    if stats is not None:
        _need(stats.is_cuda and stats.device == input.device and stats.is_contiguous() and
              stats.dtype == torch.int32 and stats.numel() == 2,
              "stats must be a contiguous int32 CUDA tensor of 2 elements on the input's device")
        sbytes = int(lib.maxk_topk_stats_scratch_bytes(n))
        scratch = torch.empty(sbytes, dtype=torch.uint8, device=input.device)
    with _device(input.device):
        check(lib.maxk_topk_cbsr_ex(_p(input), _p(sp_data), ds, _p(sp_index), is_, _p(count),
                                    _p(stats), _p(scratch), sbytes, n, d, k, TOPK_MODES[mode],
                                    _stream()), "maxk_forward")
    res = (sp_data, sp_index) if return_index else (sp_data,)
    if return_count:
        res = res + (count,)
    return res if len(res) > 1 else res[0]


def maxk_backward(grad_output: torch.Tensor, indices: torch.Tensor,
                  dim_origin: Optional[int] = None) -> torch.Tensor:
    """Dense gradient of MaxK from the ``[N, k]`` CBSR gradient.

    Reference (maxk_backward_cuda SO@0x21410): ``g = zeros(N, max(indices)+1)``;
    ``g[i, indices[i, j]] = grad_output[i, j]`` for j ascending. Checks (bindings.cpp:34-36):
    grad_output CUDA/contiguous/2-D, indices CUDA/contiguous. Here one device kernel does
    the scatter; pass ``dim_origin`` for a stable ``[N, dim_origin]`` shape (without it the
    reference's data-dependent width ``max(indices)+1`` is kept, which costs a host sync).
    """
    _need(grad_output.is_cuda, "grad_output must be a CUDA tensor")
    _need(grad_output.is_contiguous(), "grad_output must be contiguous")
    _need(grad_output.dim() == 2, "grad_output must be 2D tensor")
    _need(indices.is_cuda, "indices must be a CUDA tensor")
    _need(indices.shape == grad_output.shape, "indices must have the shape of grad_output")
    _need(grad_output.dtype == torch.float32, "grad_output must be float32")
    n, k = grad_output.shape
    # u8 selectors may be row-strided (the interleaved records of maxk_aggregate); other
    # integer dtypes are converted (contiguous)
    strided_u8 = (indices.dtype == torch.uint8 and indices.dim() == 2 and
                  (n <= 1 or indices.stride(1) == 1) and (n <= 1 or indices.stride(0) >= k))
    _need(indices.is_contiguous() or strided_u8, "indices must be contiguous")
    if indices.dtype != torch.uint8:
        _need(not indices.dtype.is_floating_point, "indices must be an integer tensor")
        indices = indices.to(torch.uint8)
    istride = indices.stride(0) if n > 1 else k
    if dim_origin is None:
        dim_origin = int(indices.max().item()) + 1 if indices.numel() else 1
    _need(1 <= k <= dim_origin <= 256, "k must be between 1 and input dimension")
    grad_in = torch.empty((n, dim_origin), dtype=torch.float32, device=grad_output.device)
    with _device(grad_output.device):
        check(lib.maxk_scatter_backward_tables(_p(grad_output), _p(indices), istride,
                                               _p(grad_in), n, dim_origin, k, _stream()),
              "maxk_backward")
    return grad_in


# -------------------------------------------------------------------------------------
# graph plans (cached partition metadata)
# -------------------------------------------------------------------------------------
class GraphPlan:
    """Owns one ``maxk_plan`` (device partition metadata for a CSR graph, k and D).

    The plan is built with ``external_workspace``: its per-call scratch (packed CBSR records,
    selector words, the two-pass E x k products) is taken from torch's caching allocator on
    the launch stream for every call, so no plan pins that memory and one plan can serve
    several streams at once. The only mutation after creation, a value refresh, is ordered
    after every earlier use on other streams (an event recorded on each of them at refresh
    time, i.e. after everything they queued) and every later use after it; calls record
    nothing (a per-call event cost ~10 us of host time on small graphs).
    """

    def __init__(self, ptr, idx, val, num_nodes, num_edges, dim_origin, dim_k,
                 num_cols: Optional[int] = None, options: Optional[dict] = None,
                 col_order: Optional[torch.Tensor] = None):
        """``options``: ``maxk_plan_options`` fields by name (``col_order`` also by name:
        'identity', 'scattered'; ``bwd_algo``: 'column_blocks', 'two_pass'); ``col_order``: an
        int32 device permutation of the columns (position -> column) for the backward's
        column blocks, which selects ``col_order='given'``."""
        self.handle = ctypes.c_void_p(0)
        self.device = ptr.device
        self._refs = (ptr, idx, val)  # keep the graph's storage alive while cached
        self.val_version = val._version if val is not None else -1
        self.num_rows = int(num_nodes)
        self.num_cols = int(num_nodes if num_cols is None else num_cols)
        self.num_edges = int(num_edges)
        self.dim_origin = int(dim_origin)
        self.dim_k = int(dim_k)
        opts = PlanOptions()
        opts.external_workspace = 1
        for key, value in (options or {}).items():
            if key in ("fwd_accumulator", "bwd_accumulator") and isinstance(value, str):
                value = ACC_KINDS[value]
            if key == "col_order" and isinstance(value, str):
                value = COL_ORDERS[value]
            if key == "bwd_algo" and isinstance(value, str):
                value = BWD_ALGOS[value]
            setattr(opts, key, int(value))
        if col_order is not None:
            _check_tensor(col_order, "col_order", torch.int32)
            _need(col_order.numel() == self.num_cols, "col_order must have num_cols entries")
            opts.col_order = COL_ORDERS["given"]
        with torch.cuda.device(ptr.device):
            check(lib.maxk_plan_create_sized(_p(ptr), _p(idx), _p(val), self.num_rows,
                                             self.num_cols, self.num_edges, self.dim_origin,
                                             self.dim_k, ctypes.byref(opts),
                                             ctypes.sizeof(opts), _p(col_order), _stream(),
                                             ctypes.byref(self.handle)), "maxk_plan_create")
        fb, bb = ctypes.c_int64(0), ctypes.c_int64(0)
        check(lib.maxk_plan_workspace_bytes(self.handle, ctypes.byref(fb), ctypes.byref(bb)),
              "maxk_plan_workspace_bytes")
        self.external = bool(opts.external_workspace)
        self.fwd_ws_bytes, self.bwd_ws_bytes = int(fb.value), int(bb.value)
        self._uses = {}        # stream id -> a stream the plan was used on
        self._refresh = None   # (stream, event) of the latest value refresh
        self._lock = threading.Lock()

    # -- stream ordering ------------------------------------------------------------------
    def _begin(self, stream):
        with self._lock:
            if self._refresh is not None and self._refresh[0] != stream:
                stream.wait_event(self._refresh[1])

    def _end(self, stream):
        sid = stream.cuda_stream
        if sid not in self._uses:
            with self._lock:
                self._uses[sid] = stream

    def _workspace(self, nbytes):
        if not self.external or nbytes == 0:
            return None, 0
        try:
            return torch.empty(nbytes, dtype=torch.uint8, device=self.device), nbytes
        except torch.OutOfMemoryError:
            # the two-pass backward's product workspace is the large one (one row chunk of
            # E x k x 4 bytes, <= 16 GiB by default, kBwdTwoPassWorkspaceCap): give the
            # allocator its cached blocks back once, then say which knob bounds it
            torch.cuda.empty_cache()
            try:
                return torch.empty(nbytes, dtype=torch.uint8, device=self.device), nbytes
            except torch.OutOfMemoryError as exc:
                raise torch.OutOfMemoryError(
                    f"maxk_kernels: per-call workspace of {nbytes} bytes does not fit; a plan "
                    f"built with options={{'bwd_tp_chunks': P}} (more row chunks) or "
                    f"{{'bwd_algo': 1}} (column blocks) needs less") from exc

    def forward(self, sp_data, sp_index, out=None, accumulate: bool = False,
                stats=None) -> torch.Tensor:
        """SpGEMM with this plan: sp tables [num_cols, k] (rows may be strided, e.g. the
        interleaved records of :mod:`maxk_kernels.dist`, gathered in place) -> out [num_rows, D];
        ``accumulate=True`` adds into the given ``out`` instead of overwriting it. ``stats``:
        fixed-point statistics covering the table instead of a pass over it, either an int32
        [n, 2] tensor of :func:`cbsr_stats` pairs or ``(tensor, n, stride)`` with pair i at
        32-bit word i * stride of the tensor's storage (the multi-GPU path keeps one pair
        per rank in a spare row of the gathered table). Without ``stats`` the call scans
        every row of the tables, so each row must be CBSR data: a ShardedAggregation's
        gathered table is not (its spare rows hold those pairs), pass its ``stats``."""
        ptr, idx, val = self._refs
        if out is None:
            if accumulate:
                raise RuntimeError("accumulate=True needs an out tensor")
            out = torch.empty((self.num_rows, self.dim_origin), dtype=torch.float32,
                              device=sp_data.device)
        stream = torch.cuda.current_stream(self.device)
        self._begin(stream)
        ws, wsb = self._workspace(self.fwd_ws_bytes)
        st, n_st, stride = None, 0, 2
        if isinstance(stats, tuple):
            st, n_st, stride = stats
            _need(st.is_cuda and st.element_size() == 4 and
                  (n_st - 1) * stride + 2 <= st.numel(), "stats does not hold n pairs")
        elif stats is not None:
            _need(stats.is_cuda and stats.is_contiguous() and stats.dtype == torch.int32 and
                  stats.dim() == 2 and stats.shape[1] == 2 and stats.shape[0] >= 1,
                  "stats must be a contiguous int32 [n, 2] CUDA tensor")
            st, n_st = stats, stats.shape[0]
        ds = _table(sp_data, "sp_data", torch.float32, self.num_cols, self.dim_k)
        is_ = _table(sp_index, "sp_index", torch.uint8, self.num_cols, self.dim_k)
        check(lib.maxk_spgemm_forward_tables(self.handle, _p(ptr), _p(idx), _p(val), _p(sp_data),
                                             ds, _p(sp_index), is_, _p(out), self.num_rows,
                                             self.num_edges, self.dim_k, self.dim_origin,
                                             int(accumulate), _p(st), n_st, stride, _p(ws), wsb,
                                             ctypes.c_void_p(stream.cuda_stream)),
              "spgemm_forward")
        self._end(stream)
        return out

    def backward(self, grad_out, sp_index, grad_sp=None) -> torch.Tensor:
        """SSpMM with this plan: grad_out [num_rows, D] -> grad_sp [num_cols, k]."""
        ptr, idx, val = self._refs
        if grad_sp is None:
            grad_sp = torch.empty((self.num_cols, self.dim_k), dtype=torch.float32,
                                  device=grad_out.device)
        stream = torch.cuda.current_stream(self.device)
        self._begin(stream)
        ws, wsb = self._workspace(self.bwd_ws_bytes)
        is_ = _table(sp_index, "sp_index", torch.uint8, self.num_cols, self.dim_k)
        check(lib.maxk_sspmm_backward_tables(self.handle, _p(ptr), _p(idx), _p(val),
                                             _p(grad_out), _p(sp_index), is_, _p(grad_sp),
                                             self.num_rows, self.num_edges, self.dim_k,
                                             self.dim_origin, _p(ws), wsb,
                                             ctypes.c_void_p(stream.cuda_stream)),
              "spgemm_backward")
        self._end(stream)
        return grad_sp

    def refresh_values(self, val: torch.Tensor) -> None:
        """Re-snapshot in-place-modified edge values (same tensor, new ``_version``); runs
        after every earlier use of the plan on any stream."""
        stream = torch.cuda.current_stream(self.device)
        with self._lock:
            for other in self._uses.values():
                if other != stream:  # after everything queued on it so far
                    ev = torch.cuda.Event()
                    ev.record(other)
                    stream.wait_event(ev)
        with torch.cuda.device(self.device):
            check(lib.maxk_plan_refresh_values(self.handle, _p(val),
                                               ctypes.c_void_p(stream.cuda_stream)),
                  "maxk_plan_refresh_values")
        ev = torch.cuda.Event()
        ev.record(stream)
        with self._lock:
            self._refresh = (stream, ev)
            self._uses[stream.cuda_stream] = stream
        self._refs = (self._refs[0], self._refs[1], val)
        self.val_version = val._version

    def info(self) -> dict:
        info = PlanInfo()
        check(lib.maxk_plan_get_info_sized(self.handle, ctypes.byref(info), ctypes.sizeof(info)),
              "maxk_plan_get_info")
        d = info.as_dict()
        d["fwd_workspace_bytes"] = self.fwd_ws_bytes
        d["bwd_workspace_bytes"] = self.bwd_ws_bytes
        return d

    @property
    def device_bytes(self) -> int:
        return int(self.info()["device_bytes"])

    def new_cbsr(self):
        """Uninitialised ``(sp_data, sp_index)`` [num_cols, k] tables in the layout this plan's
        forward gathers (``fwd_layout``): strided views of one buffer of packed records
        (``fwd_record_bytes`` per column, values then selectors) when the forward reads packed
        records, so a top-k written there (:func:`maxk_forward` ``out=``) needs no per-call
        pack; two plain tables otherwise."""
        layout = getattr(self, "_layout", None)
        if layout is None:
            info = self.info()
            layout = self._layout = (info["fwd_layout"], info["fwd_record_bytes"])
        n, k = self.num_cols, self.dim_k
        if layout[0] == 1 and n > 0:
            rec = torch.empty((n, layout[1]), dtype=torch.uint8, device=self.device)
            return rec[:, :4 * k].view(torch.float32), rec[:, 4 * k:5 * k]
        return (torch.empty((n, k), dtype=torch.float32, device=self.device),
                torch.empty((n, k), dtype=torch.uint8, device=self.device))

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value and lib is not None:
            lib.maxk_plan_destroy(h)
            self.handle = ctypes.c_void_p(0)


# Plans are cached per (graph structure, edge-value tensor, k, D): two value sets on one
# structure (SAGE 'mean' and GCN 'both' weights, say) get two plans instead of refreshing
# one plan back and forth. The cache is bounded by the device memory the plans hold
# (MAXK_PLAN_CACHE_BYTES, default a quarter of the device's HBM: ~72 GB on MI355X, twenty
# Reddit-sized plans) and by a count.
_PLAN_CACHE: "collections.OrderedDict[tuple, GraphPlan]" = collections.OrderedDict()
_PLAN_CACHE_SIZE = 32
_PLAN_CACHE_BYTES: Optional[int] = (int(os.environ["MAXK_PLAN_CACHE_BYTES"])
                                    if "MAXK_PLAN_CACHE_BYTES" in os.environ else None)
_PLAN_LOCK = threading.Lock()


def _cache_budget(device) -> int:
    if _PLAN_CACHE_BYTES is not None:
        return _PLAN_CACHE_BYTES
    return torch.cuda.get_device_properties(device).total_memory // 4


def get_plan(ptr, idx, val, num_nodes, num_edges, dim_origin, dim_k) -> GraphPlan:
    """Cached plan for (graph storage, structure version, value tensor, k, D); in-place
    edits of ``val`` (a new ``val._version``) refresh the plan's value snapshot."""
    key = (ptr.device.index, ptr.data_ptr(), idx.data_ptr(), ptr._version, idx._version,
           val.data_ptr(), int(num_nodes), int(num_edges), int(dim_origin), int(dim_k))
    with _PLAN_LOCK:
        plan = _PLAN_CACHE.get(key)
        if plan is not None:
            _PLAN_CACHE.move_to_end(key)
            if plan._refs[2] is not val or plan.val_version != val._version:
                plan.refresh_values(val)
            return plan
        plan = GraphPlan(ptr, idx, val, int(num_nodes), int(num_edges), int(dim_origin),
                         int(dim_k))
        _PLAN_CACHE[key] = plan
        budget = _cache_budget(ptr.device)
        total = sum(p.device_bytes for p in _PLAN_CACHE.values())
        while len(_PLAN_CACHE) > 1 and (len(_PLAN_CACHE) > _PLAN_CACHE_SIZE or total > budget):
            _, old = _PLAN_CACHE.popitem(last=False)
            total -= old.device_bytes
        return plan


def cached_plan_bytes() -> int:
    with _PLAN_LOCK:
        return sum(p.device_bytes for p in _PLAN_CACHE.values())


def clear_plan_cache() -> None:
    with _PLAN_LOCK:
        _PLAN_CACHE.clear()


def _check_graph(ptr, idx, val, num_nodes, num_edges):
    _check_tensor(ptr, "ptr", torch.int32)
    _check_tensor(idx, "idx", torch.int32)
    _check_tensor(val, "val", torch.float32)
    _need(ptr.dim() == 1 and ptr.numel() == num_nodes + 1, "ptr must have num_nodes+1 entries")
    _need(idx.numel() == num_edges and val.numel() == num_edges,
          "idx and val must have num_edges entries")


# -------------------------------------------------------------------------------------
# SpGEMM forward / SSpMM backward
# -------------------------------------------------------------------------------------
def spgemm_forward(ptr, idx, val, sp_data, sp_index, num_nodes: int, num_edges: int,
                   dim_k: int, dim_origin: int, plan: Optional[GraphPlan] = None
                   ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Row-wise-product SpGEMM over CBSR features.

    Reference ``spgemm_forward(ptr, idx, val, sp_data, sp_index, num_nodes, num_edges,
    dim_k, dim_origin) -> (out[num_nodes, dim_origin], sp_index)`` (spgemm_forward_cuda
    SO@0x221a0; checks bindings.cpp:45-54): ``out[r] = sum_nz val[nz] *
    densify(sp_data[idx[nz]], sp_index[idx[nz]])``.
    """
    if plan is None or plan._refs[0] is not ptr or plan._refs[1] is not idx or plan._refs[2] is not val:
        _check_graph(ptr, idx, val, num_nodes, num_edges)  # (a plan's own tensors were checked)
    _check_tensor(sp_data, "sp_data", torch.float32)
    _check_tensor(sp_index, "sp_index", torch.uint8)
    _need(sp_data.shape == (num_nodes, dim_k) and sp_index.shape == (num_nodes, dim_k),
          "sp_data and sp_index must be [num_nodes, dim_k]")
    _need(1 <= dim_k <= dim_origin <= 256, "k must be between 1 and input dimension")
    if plan is None:
        plan = get_plan(ptr, idx, val, num_nodes, num_edges, dim_origin, dim_k)
    _need(plan.num_rows == num_nodes and plan.num_edges == num_edges and
          plan.dim_k == dim_k and plan.dim_origin == dim_origin,
          "plan was built for a different graph / k / D")
    with _device(sp_data.device):
        out = plan.forward(sp_data, sp_index)
    return out, sp_index


def spgemm_backward(ptr, idx, val, grad_output, sp_index, num_nodes: int, num_edges: int,
                    dim_k: int, dim_origin: int, plan: Optional[GraphPlan] = None
                    ) -> torch.Tensor:
    """Outer-product SSpMM: ``grad_sp[c, l] = sum_{(r,c)} val * grad_output[r, sp_index[c, l]]``.

    Reference ``spgemm_backward(ptr, idx, val, grad_output, sp_index, num_nodes,
    num_edges, dim_k, dim_origin) -> [num_nodes, dim_k]`` (spgemm_backward_cuda
    SO@0x22490; checks bindings.cpp:65-71).
    """
    if plan is None or plan._refs[0] is not ptr or plan._refs[1] is not idx or plan._refs[2] is not val:
        _check_graph(ptr, idx, val, num_nodes, num_edges)
    _check_tensor(grad_output, "grad_output", torch.float32)
    _check_tensor(sp_index, "sp_index", torch.uint8)
    _need(grad_output.shape == (num_nodes, dim_origin), "grad_output must be [num_nodes, dim_origin]")
    _need(sp_index.shape == (num_nodes, dim_k), "sp_index must be [num_nodes, dim_k]")
    _need(1 <= dim_k <= dim_origin <= 256, "k must be between 1 and input dimension")
    if plan is None:
        plan = get_plan(ptr, idx, val, num_nodes, num_edges, dim_origin, dim_k)
    _need(plan.num_rows == num_nodes and plan.num_edges == num_edges and
          plan.dim_k == dim_k and plan.dim_origin == dim_origin,
          "plan was built for a different graph / k / D")
    with _device(grad_output.device):
        grad_sp = plan.backward(grad_output, sp_index)
    return grad_sp


def plan_col_order(plan: GraphPlan) -> torch.Tensor:
    """The plan's column order: int32 [num_cols], position -> column of the backward's column
    blocks (the identity for plans without one)."""
    out = torch.empty(plan.num_cols, dtype=torch.int32, device=plan.device)
    with torch.cuda.device(plan.device):
        check(lib.maxk_plan_get_col_order(plan.handle, _p(out), _stream()), "plan_col_order")
    return out


def cbsr_stats(sp_data: torch.Tensor, sp_index: torch.Tensor,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Fixed-point statistics of a CBSR table (``maxk_cbsr_stats``): int32 [1, 2] (written
    into ``out`` when given), the pair :meth:`GraphPlan.forward` takes as ``stats``."""
    _need(sp_data.dim() == 2 and sp_index.shape == sp_data.shape,
          "sp_data and sp_index must be [N, k]")
    n, k = sp_data.shape
    ds = _table(sp_data, "sp_data", torch.float32, n, k)
    is_ = _table(sp_index, "sp_index", torch.uint8, n, k)
    if out is None:
        out = torch.empty((1, 2), dtype=torch.int32, device=sp_data.device)
    _need(out.is_cuda and out.is_contiguous() and out.dtype == torch.int32 and out.numel() == 2,
          "out must be a contiguous int32 CUDA tensor of 2 elements")
    with torch.cuda.device(sp_data.device):
        check(lib.maxk_cbsr_stats_tables(_p(sp_data), ds, _p(sp_index), is_, n, k, _p(out),
                                         _stream()), "cbsr_stats")
    return out


def dense_spmm(ptr, idx, val, x) -> torch.Tensor:
    """Dense CSR SpMM comparator (DGL ``update_all(copy_u, sum)`` with edge weights). The
    kernel takes float4 rows: other widths run on a copy padded to a multiple of 4 features
    (zeros; DGL's SAGEConv/GraphConv/GINConv accept any hidden size)."""
    _check_tensor(x, "x", torch.float32)
    _check_graph(ptr, idx, val, x.shape[0], idx.numel())
    _need(x.dim() == 2, "x must be 2D")
    d = x.shape[1]
    d4 = (d + 3) // 4 * 4
    xin = x if d4 == d else torch.nn.functional.pad(x, (0, d4 - d)).contiguous()
    y = torch.empty_like(xin)
    with torch.cuda.device(x.device):
        check(lib.maxk_dense_spmm_csr(_p(ptr), _p(idx), _p(val), _p(xin), _p(y), x.shape[0],
                                      d4, _stream()), "dense_spmm")
    return y if d4 == d else y[:, :d].contiguous()
