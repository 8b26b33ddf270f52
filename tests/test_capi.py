"""CPU: the C-ABI library loads, exports every declared symbol, and rejects bad arguments
on the host (no compute call reaches a GPU here)."""
import ctypes
import os
import re

import numpy as np
import pytest

import maxk_kernels
from maxk_kernels import _lib
from oracle import oracle
from maxk_kernels import graphs, warp4

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "maxk_hip.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(maxk_\w+)\s*\(", text)))


def test_library_is_in_tree_and_loaded():
    assert os.path.exists(_lib.LIB_PATH)
    assert _lib.LIB_PATH.startswith(os.path.join(ROOT, "spgemm-gnn_amd"))
    assert maxk_kernels.ABI_VERSION == 4


def test_exports_every_declared_symbol():
    names = declared_functions()
    assert len(names) >= 12
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for n in names:
        assert hasattr(lib, n), n
    # and the ctypes binding covers exactly the header
    assert set(names) == set(_lib.SIGNATURES)


def test_library_targets_gfx950():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


@pytest.mark.parametrize("args", [
    (0, 256, 16, 0),      # ok size-0 -> MAXK_OK without touching the GPU
])
def test_topk_zero_rows_is_noop(args):
    n, d, k, mode = args
    assert _lib.lib.maxk_topk_cbsr(None, None, None, n, d, k, mode, None) == 0


@pytest.mark.parametrize("n,d,k,mode,expect", [
    (10, 256, 0, 0, -1),    # k < 1
    (10, 256, 257, 0, -1),  # k > D
    (10, 300, 8, 0, -1),    # D > 256 (u8 selectors)
    (10, 256, 8, 7, -1),    # unknown mode
    (10, 256, 8, 0, -1),    # null pointers
])
def test_topk_argument_errors(n, d, k, mode, expect):
    rc = _lib.lib.maxk_topk_cbsr(None, None, None, n, d, k, mode, None)
    assert rc == expect
    msg = _lib.lib.maxk_last_error().decode()
    assert msg


def test_reference_error_message_for_k():
    _lib.lib.maxk_topk_cbsr(None, None, None, 4, 64, 65, 0, None)
    assert "k must be between 1 and input dimension" in _lib.lib.maxk_last_error().decode()


def test_plan_create_argument_errors():
    h = ctypes.c_void_p(0)
    assert _lib.lib.maxk_plan_create(None, None, None, 10, 100, 256, 16, None,
                                     ctypes.byref(h)) == -1
    assert _lib.lib.maxk_plan_create(None, None, None, 10, 100, 256, 300, None,
                                     ctypes.byref(h)) == -1
    assert _lib.lib.maxk_plan_create(None, None, None, 10, 100, 256, 16, None, None) == -1
    assert not h.value


def test_spgemm_rejects_null_plan():
    rc = _lib.lib.maxk_spgemm_forward(None, None, None, None, None, None, None, 10, 100, 16,
                                      256, None)
    assert rc == -1


def test_warp4_build_matches_oracle():
    ptr, _ = graphs.synthetic_csr(700, 30_000, seed=3)
    t = warp4.build_warp4(ptr)
    assert np.array_equal(t, oracle.warp4(ptr.numpy()))
    # the reference's consumer derives num_warps = bytes / 16 and grid = ceil(W / 12)
    assert t.shape[1] == 4 and (t[:, 3] == 0).all() and (t[:, 2] <= 64).all()


def test_warp4_file_roundtrip(tmp_path):
    ptr, _ = graphs.synthetic_csr(100, 2000, seed=4)
    t = warp4.build_warp4(ptr)
    p = warp4.warp4_path("graph", str(tmp_path))
    warp4.write_warp4(p, t)
    assert os.path.getsize(p) == t.size * 4
    assert np.array_equal(warp4.read_warp4(p), t)


def test_warp4_replay_validates_against_ptr(tmp_path):
    """A reference-generated .warp4 (here: the oracle's chunk rule, the reference's
    generate_meta.py being absent) replays against ptr; a stale or corrupt one is refused."""
    ptr, _ = graphs.synthetic_csr(300, 9000, seed=5)
    hp = ptr.numpy()
    t = oracle.warp4(hp)
    warp4.write_warp4(warp4.warp4_path("graph", str(tmp_path)), t)
    got = warp4.replay_warp4(ptr, "graph", str(tmp_path), strict=True)
    assert np.array_equal(got, t)
    assert np.array_equal(warp4.ptr_from_warp4(t, hp.size - 1), hp)
    # any other exact tiling (shuffled entries, 32-nz chunks) sums the same nonzeros
    warp4.validate_warp4(t[np.random.default_rng(0).permutation(len(t))], ptr)
    t32 = oracle.warp4(hp, max_nz=32)
    warp4.validate_warp4(t32, ptr)
    with pytest.raises(ValueError, match="canonical"):
        warp4.validate_warp4(t32, ptr, strict=True)
    # the graph with one more edge in row 7: the table no longer matches
    other = hp.copy()
    other[8:] += 1
    with pytest.raises(ValueError, match="does not match ptr"):
        warp4.validate_warp4(t, other)
    bad = t.copy(); bad[3, 3] = 1
    with pytest.raises(ValueError, match="4th word"):
        warp4.validate_warp4(bad, ptr)
    bad = t.copy(); bad[5, 1] += 1
    with pytest.raises(ValueError, match="gap or overlap|first chunk"):
        warp4.validate_warp4(bad, ptr)
    bad = t.copy(); bad[2, 2] = 65
    with pytest.raises(ValueError, match="length"):
        warp4.validate_warp4(bad, ptr)
    with pytest.raises(ValueError, match="row out of range"):
        warp4.ptr_from_warp4(t, 10)
    assert np.array_equal(warp4.ptr_from_warp4(np.zeros((0, 4), np.int32), 3), [0, 0, 0, 0])


def test_python_checks_mirror_reference_messages():
    import torch
    x = torch.zeros(4, 8)
    with pytest.raises(RuntimeError, match="input must be a CUDA tensor"):
        maxk_kernels.maxk_forward(x, 2)


def test_baseline_library_exports_its_header():
    header = os.path.join(ROOT, "include", "maxk_baseline.h")
    text = re.sub(r"/\*.*?\*/", "", open(header).read(), flags=re.S)
    names = sorted(set(re.findall(r"\b(maxk_\w+)\s*\(", text)))
    assert names == ["maxk_baseline_last_error", "maxk_spmm_rocsparse",
                     "maxk_spmm_rocsparse_coo"]
    lib = ctypes.CDLL(os.path.join(os.path.dirname(_lib.LIB_PATH), "libmaxk_baseline.so"))
    for n in names:
        assert hasattr(lib, n), n
    from maxk_kernels import baselines
    bl = baselines._lib()
    ms = ctypes.c_float()
    assert bl.maxk_spmm_rocsparse(None, None, None, None, None, -1, 0, 8, 0, 0,
                                  ctypes.byref(ms), None) == -1
    assert bl.maxk_spmm_rocsparse_coo(None, None, None, None, None, 4, -1, 8, 0, 0,
                                      ctypes.byref(ms), None) == -1
    assert b"maxk_spmm_rocsparse_coo" in bl.maxk_baseline_last_error()


def _struct_fields(name):
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    body = re.search(r"typedef struct " + name + r"\s*\{(.*?)\}\s*" + name + ";", text, re.S)
    fields = []
    for decl in body.group(1).split(";"):
        m = re.search(r"\b(int32_t|int64_t)\s+(\w+)(\[(\d+)\])?\s*$", decl.strip())
        if m:
            fields.append((m.group(2), m.group(1), int(m.group(4) or 1)))
    return fields


@pytest.mark.parametrize("cname,pycls", [("maxk_plan_options", "PlanOptions"),
                                          ("maxk_plan_info", "PlanInfo")])
def test_ctypes_structs_mirror_header(cname, pycls):
    """The ctypes mirrors must match the C structs field by field (names, widths, order)."""
    fields = _struct_fields(cname)
    py = getattr(_lib, pycls)._fields_
    assert [f[0] for f in fields] == [f[0] for f in py]
    for (name, ctype, count), (_, pytype) in zip(fields, py):
        width = 4 if ctype == "int32_t" else 8
        assert ctypes.sizeof(pytype) == width * count, name


def test_header_is_plain_c(tmp_path):
    """include/maxk_hip.h is the drop-in boundary for any FFI: it must compile as C99 on its
    own (no C++, no HIP or torch types)."""
    import shutil
    import subprocess
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    src = tmp_path / "use_header.c"
    src.write_text('#include "maxk_hip.h"\n'
                   "int main(void) {\n"
                   "  maxk_plan_options o = {0};\n"
                   "  maxk_plan_info i;\n"
                   "  (void)o; (void)i;\n"
                   "  return maxk_abi_version() == MAXK_ABI_VERSION ? 0 : 1;\n"
                   "}\n")
    r = subprocess.run([cc, "-std=c99", "-Wall", "-Werror", "-pedantic", "-fsyntax-only",
                        "-I", os.path.dirname(HEADER), str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_plan_create_sized_option_sizes():
    """maxk_plan_create_sized reads opts_bytes of the caller's options: a smaller (older)
    struct leaves the rest at 0, a larger (newer) one must have its extra fields at 0, and the
    size must be whole int32 fields. All rejected on the host, before any device call."""
    opts = _lib.PlanOptions()
    size = ctypes.sizeof(opts)
    h = ctypes.c_void_p(0)
    lib = _lib.lib
    args = (None, None, None, 10, 10, 100, 256, 16)
    assert lib.maxk_plan_create_sized(*args, ctypes.byref(opts), 6, None, None,
                                      ctypes.byref(h)) == -1
    assert "multiple of 4" in lib.maxk_last_error().decode()
    bigger = (ctypes.c_uint8 * (size + 8))()
    bigger[size + 4] = 1                              # a field this library does not know
    assert lib.maxk_plan_create_sized(*args, ctypes.cast(bigger, ctypes.c_void_p), size + 8,
                                      None, None, ctypes.byref(h)) == -1
    assert "newer" in lib.maxk_last_error().decode()
    bigger[size + 4] = 0                              # zero extra fields are accepted ...
    assert lib.maxk_plan_create_sized(*args, ctypes.cast(bigger, ctypes.c_void_p), size + 8,
                                      None, None, ctypes.byref(h)) == -1
    assert "null pointer" in lib.maxk_last_error().decode()   # ... then ptr = NULL is refused
    # create_ex reads the round-1 layout: 120 bytes, up to fwd_rot_rate; external_workspace ..
    # bwd_tp_store (offsets 120..143) and the ABI-2 fields only through create_sized
    assert _lib.PlanOptions.bwd_flush.offset == 31 * 4 and _lib.PlanOptions.external_workspace.offset == 120
    assert _lib.PlanOptions.bwd_row_cost.offset == 144
    # an ABI-2 option (col_order = 4) needs the permutation argument
    opts.col_order = 4
    assert lib.maxk_plan_create_sized(*args, ctypes.byref(opts), size, None, None,
                                      ctypes.byref(h)) == -1
    assert "col_order" in lib.maxk_last_error().decode()
    assert not h.value
    info = _lib.PlanInfo()
    assert lib.maxk_plan_get_info_sized(None, ctypes.byref(info), ctypes.sizeof(info)) == -1


def _header_enum(prefix):
    text = open(HEADER).read()
    return {m.group(1): int(m.group(2))
            for m in re.finditer(r"\b(" + prefix + r"\w+)\s*=\s*(-?\d+)", text)}


def test_header_enums_match_binding():
    """The documented enumerations the library writes into maxk_plan_info (col_order, bwd_algo)
    and reads from the options equal the Python binding's name tables."""
    co = _header_enum("MAXK_COL_ORDER_")
    assert {k.replace("MAXK_COL_ORDER_", "").lower(): v for k, v in co.items()} == _lib.COL_ORDERS
    ba = _header_enum("MAXK_BWD_")
    assert {k.replace("MAXK_BWD_", "").lower(): v for k, v in ba.items()} == _lib.BWD_ALGOS
    v1 = int(re.search(r"#define MAXK_PLAN_OPTIONS_V1_BYTES (\d+)", open(HEADER).read()).group(1))
    assert v1 == _lib.PlanOptions.external_workspace.offset == 120


def test_removed_options_refused_on_host():
    """ABI 3: option values of removed kernel organisations are refused before any device
    call, with MAXK_ERR_UNSUPPORTED and a message naming the option."""
    lib = _lib.lib
    h = ctypes.c_void_p(0)
    for name, value in (("col_order", 3), ("bwd_algo", 2), ("fwd_persistent", 1),
                        ("bwd_features_per_lane", 1), ("quad_loads", 2)):
        opts = _lib.PlanOptions()
        setattr(opts, name, value)
        rc = lib.maxk_plan_create_sized(None, None, None, 10, 10, 100, 256, 16, ctypes.byref(opts),
                                        ctypes.sizeof(opts), None, None, ctypes.byref(h))
        assert rc == -2, name
        msg = lib.maxk_last_error().decode()
        assert "removed in ABI 3" in msg and name.split("_")[0] in msg, msg
    assert not h.value


def test_create_ex_reads_only_the_round1_layout():
    """maxk_plan_create_ex reads the 120 bytes of its round-1 options layout and no
    more. A 120-byte buffer followed by bytes that would be invalid options (external_workspace
    = 7, bwd_flush = 9) is not read past: the call fails on the null graph pointer, not on an
    option. The same bytes through create_sized with the full size are read and refused."""
    lib = _lib.lib
    h = ctypes.c_void_p(0)
    size = ctypes.sizeof(_lib.PlanOptions)
    buf = (ctypes.c_int32 * (size // 4))()
    buf[120 // 4] = 7          # external_workspace
    buf[124 // 4] = 9          # bwd_flush
    args = (None, None, None, 10, 10, 100, 256, 16)
    rc = lib.maxk_plan_create_ex(*args, ctypes.cast(buf, ctypes.c_void_p), None, ctypes.byref(h))
    assert rc == -1 and "null pointer" in lib.maxk_last_error().decode()
    rc = lib.maxk_plan_create_sized(*args, ctypes.cast(buf, ctypes.c_void_p), size, None, None,
                                    ctypes.byref(h))
    assert rc == -1 and "external_workspace" in lib.maxk_last_error().decode()
    assert not h.value


def test_backward_shapes_without_a_kernel_refused_on_host():
    """ABI 4: an explicit bwd_unroll that the explicit bwd_waves has no kernel for
    (16 waves run 8 sub-steps only; 12 waves 8 or 12) is refused with MAXK_ERR_INVALID_ARG
    before any device call, instead of being replaced by 8; the combinations that exist pass
    the option checks (and then fail on the null graph)."""
    lib = _lib.lib
    h = ctypes.c_void_p(0)
    for waves, unroll, ok in ((16, 12, False), (16, 16, False), (12, 16, False), (16, 8, True),
                              (12, 12, True), (12, 8, True), (8, 16, True), (8, 12, True),
                              (0, 16, True), (0, 12, True)):
        opts = _lib.PlanOptions()
        opts.bwd_waves, opts.bwd_unroll = waves, unroll
        rc = lib.maxk_plan_create_sized(None, None, None, 10, 10, 100, 256, 16, ctypes.byref(opts),
                                        ctypes.sizeof(opts), None, None, ctypes.byref(h))
        msg = lib.maxk_last_error().decode()
        assert rc == -1, (waves, unroll)
        assert ("bwd_waves" in msg) != ok, (waves, unroll, msg)
    assert not h.value


def test_topk_stats_scratch_contract():
    """maxk_topk_cbsr_ex with stats needs maxk_topk_stats_scratch_bytes(N) of scratch: one
    8-B partial pair per 4 rows (per wave of the exact kernel, per work-group of the
    ref_compat one), refused on the host when smaller or missing."""
    lib = _lib.lib
    assert lib.maxk_topk_stats_scratch_bytes(0) == 64
    assert lib.maxk_topk_stats_scratch_bytes(16) == 8 * 4 + 64
    assert lib.maxk_topk_stats_scratch_bytes(17) == 8 * 8 + 64
    P = ctypes.c_void_p
    n = 100
    need = lib.maxk_topk_stats_scratch_bytes(n)
    for scratch, nbytes in ((None, need), (P(16), need - 1)):
        rc = lib.maxk_topk_cbsr_ex(P(16), P(16), 0, P(16), 0, None, P(16), scratch, nbytes, n,
                                   256, 16, 0, None)
        assert rc == -1 and "scratch" in lib.maxk_last_error().decode()
