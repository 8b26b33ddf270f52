"""GPU fuzz parity: random small graphs, widths and k through the four reference functions,
against the CPU oracle (hypothesis, derandomized so every run draws the same cases).

Each example draws a CSR (empty rows, heavy rows, repeated and unsorted columns allowed),
a feature width D in [1, 256] and k in [1, D], and checks: the top-k bit for bit (both
modes), the SpGEMM forward and the SSpMM backward within the fp32-accumulator bar, and the
MaxK scatter exactly.
"""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import maxk_kernels as mk
from oracle import oracle

pytestmark = pytest.mark.gpu

_RAN = []  # cases of the option fuzz that ran to completion


def _graph(rs, n, avg_deg, heavy, unsorted, repeats):
    deg = rs.poisson(avg_deg, n).astype(np.int64)
    if heavy and n > 1:
        deg[rs.randint(n)] = rs.randint(n, 6 * n)      # a row split over forward tasks
    cols = []
    for r in range(n):
        c = rs.randint(0, n, deg[r]).astype(np.int32)
        if not repeats:
            c = np.unique(c)
        if not unsorted:
            c = np.sort(c)
        cols.append(c)
    ptr = np.zeros(n + 1, np.int32)
    ptr[1:] = np.cumsum([c.size for c in cols])
    idx = np.concatenate(cols).astype(np.int32) if cols else np.zeros(0, np.int32)
    val = rs.randn(idx.size).astype(np.float32)
    return ptr, idx, val


@settings(max_examples=150, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(n=st.integers(1, 2500), avg_deg=st.sampled_from([0.0, 0.5, 3.0, 20.0, 60.0]),
       d=st.integers(1, 256), kfrac=st.floats(0.0, 1.0), heavy=st.booleans(),
       unsorted=st.booleans(), repeats=st.booleans(), seed=st.integers(0, 2**31 - 1))
def test_random_graph_vs_oracle(gpu, n, avg_deg, d, kfrac, heavy, unsorted, repeats, seed):
    rs = np.random.RandomState(seed)
    k = max(1, min(d, int(round(kfrac * d))))
    p, ix, v = _graph(rs, n, avg_deg, heavy, unsorted, repeats)
    x = rs.randn(n, d).astype(np.float32)
    g = rs.randn(n, d).astype(np.float32)
    xt = torch.from_numpy(x).to(gpu)
    for mode in ("exact", "ref_compat"):
        sd, si = mk.maxk_forward(xt, k, mode=mode, return_index=True)
        od, oi = oracle.maxk(x, k, mode)
        assert np.array_equal(si.cpu().numpy(), oi), mode
        assert np.array_equal(sd.cpu().numpy().view(np.uint32), od.view(np.uint32)), mode
    od, oi = oracle.maxk(x, k, "exact")
    ptr, idx, val = (torch.from_numpy(a).to(gpu) for a in (p, ix, v))
    sd, si = torch.from_numpy(od).to(gpu), torch.from_numpy(oi).to(gpu)
    out, _ = mk.spgemm_forward(ptr, idx, val, sd, si, n, ix.size, k, d)
    ref, mag = oracle.spgemm_forward(p, ix, v, od, oi, d, with_mag=True)
    ok, worst = oracle.close_enough(out.cpu().numpy(), ref, mag)
    assert ok, ("forward", worst)
    gs = mk.spgemm_backward(ptr, idx, val, torch.from_numpy(g).to(gpu), si, n, ix.size, k, d)
    ref, mag = oracle.sspmm_backward(p, ix, v, g, oi, with_mag=True)
    ok, worst = oracle.close_enough(gs.cpu().numpy(), ref, mag)
    assert ok, ("backward", worst)
    gin = mk.maxk_backward(gs, si, dim_origin=d)
    assert np.array_equal(gin.cpu().numpy(), oracle.maxk_backward(gs.cpu().numpy(), oi, d))
    mk.clear_plan_cache()


@settings(max_examples=100, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture,
                                 HealthCheck.filter_too_much])
@given(n=st.integers(1, 1500), avg_deg=st.sampled_from([0.0, 0.5, 3.0, 20.0, 60.0]),
       d=st.integers(1, 256), kfrac=st.floats(0.0, 1.0), heavy=st.booleans(),
       opt=st.integers(0, 10_000), seed=st.integers(0, 2**31 - 1))
def test_random_graph_plan_options_vs_oracle(gpu, n, avg_deg, d, kfrac, heavy, opt, seed):
    """The same draws through a plan built with one of the parity tests' option sets
    (tests/test_gpu_parity.py PLAN_OPTIONS). Every such set is valid for every (graph, D, k)
    since ABI 3 (k is padded to whole lanes, slot groups shrink to divide it, a two-pass
    request falls back to column blocks where k / 4 is not a power of two): a plan-creation
    error fails the case instead of being assumed away, so all drawn cases run."""
    from test_gpu_parity import PLAN_OPTIONS
    opts = PLAN_OPTIONS[opt % len(PLAN_OPTIONS)]
    rs = np.random.RandomState(seed)
    k = max(1, min(d, int(round(kfrac * d))))
    p, ix, v = _graph(rs, n, avg_deg, heavy, unsorted=bool(seed & 1), repeats=bool(seed & 2))
    x = rs.randn(n, d).astype(np.float32)
    g = rs.randn(n, d).astype(np.float32)
    od, oi = oracle.maxk(x, k, "exact")
    ptr, idx, val = (torch.from_numpy(a).to(gpu) for a in (p, ix, v))
    plan = mk.GraphPlan(ptr, idx, val, n, ix.size, d, k, options=opts)
    _RAN.append((n, d, k, opt % len(PLAN_OPTIONS)))
    out = plan.forward(torch.from_numpy(od).to(gpu), torch.from_numpy(oi).to(gpu))
    ref, mag = oracle.spgemm_forward(p, ix, v, od, oi, d, with_mag=True)
    ok, worst = oracle.close_enough(out.cpu().numpy(), ref, mag)
    assert ok, ("forward", opts, worst)
    gs = plan.backward(torch.from_numpy(g).to(gpu), torch.from_numpy(oi).to(gpu))
    ref, mag = oracle.sspmm_backward(p, ix, v, g, oi, with_mag=True)
    ok, worst = oracle.close_enough(gs.cpu().numpy(), ref, mag)
    assert ok, ("backward", opts, worst)


def test_option_fuzz_ran_every_case(gpu):
    """Runs after the option fuzz (file order): hypothesis drew 100 cases and none was skipped
    (derandomized draws: the same cases every run)."""
    if not _RAN:
        pytest.skip("the option fuzz did not run in this session (-k selection)")
    assert len(_RAN) >= 100, len(_RAN)
    print(f"option fuzz: {len(_RAN)} cases, {len(set(c[3] for c in _RAN))} option sets, "
          f"k in [{min(c[2] for c in _RAN)}, {max(c[2] for c in _RAN)}]")
