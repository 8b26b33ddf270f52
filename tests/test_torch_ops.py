"""torch.ops.maxk.* registration (maxk_kernels/torch_ops.py; VERDICT r04 weak 9: the
reference's pybind11 extension, /root/reference/setup.py:23-24, is opaque to torch tooling).

CPU: the schemas exist, the fake kernels give the reference's output shapes, a MaxK +
SpGEMM layer traces through ``make_fx`` as one node per call, and autograd through the fake
kernels reaches the registered derivatives (``maxk_backward``, ``spgemm_backward``).
GPU: ``torch.library.opcheck`` on every operator, and ``torch.compile(fullgraph=True)`` of a
MaxK layer step equal to the eager step (which the parity suites check against the oracle).
"""
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode
from torch.fx.experimental.proxy_tensor import make_fx

import maxk_kernels as mk
from maxk_kernels import graphs

OPS = ("maxk_forward", "maxk_backward", "spgemm_forward", "spgemm_backward")


def _graph(n, e, dev, seed=3):
    ptr, idx = graphs.synthetic_csr(n, e, seed=seed)
    ptr, idx = ptr.to(dev), idx.to(dev)
    val = torch.rand(idx.numel(), generator=torch.Generator().manual_seed(seed)).to(dev)
    return ptr, idx, val


def _layer(ptr, idx, val, x, k):
    n, d = x.shape
    sp_data, sp_index = torch.ops.maxk.maxk_forward(x, k)
    return torch.ops.maxk.spgemm_forward(ptr, idx, val, sp_data, sp_index, n, idx.numel(), k, d)


# ------------------------------------------------------------------------ CPU
def test_operators_are_registered():
    for name in OPS:
        op = getattr(torch.ops.maxk, name)
        assert op.default._schema.name == f"maxk::{name}"


def test_fake_kernels_give_reference_shapes():
    with FakeTensorMode():
        x = torch.empty(50, 64, device="cuda")
        sp_data, sp_index = torch.ops.maxk.maxk_forward(x, 16)
        assert sp_data.shape == (50, 16) and sp_data.dtype == torch.float32
        assert sp_index.shape == (50, 16) and sp_index.dtype == torch.uint8
        g = torch.ops.maxk.maxk_backward(sp_data, sp_index, 64)
        assert g.shape == (50, 64)
        ptr = torch.empty(51, dtype=torch.int32, device="cuda")
        idx = torch.empty(300, dtype=torch.int32, device="cuda")
        val = torch.empty(300, device="cuda")
        out = torch.ops.maxk.spgemm_forward(ptr, idx, val, sp_data, sp_index, 50, 300, 16, 64)
        assert out.shape == (50, 64) and out.device.type == "cuda"
        gs = torch.ops.maxk.spgemm_backward(ptr, idx, val, out, sp_index, 50, 300, 16, 64)
        assert gs.shape == (50, 16)


def test_layer_traces_as_one_node_per_call():
    with FakeTensorMode() as mode:
        ptr = mode.from_tensor(torch.zeros(41, dtype=torch.int32)).to("cuda")
        idx = torch.empty(200, dtype=torch.int32, device="cuda")
        val = torch.empty(200, device="cuda")
        x = torch.empty(40, 32, device="cuda")
        gm = make_fx(lambda p, i, v, h: _layer(p, i, v, h, 8), tracing_mode="fake")(ptr, idx, val, x)
    targets = [str(n.target) for n in gm.graph.nodes if n.op == "call_function"]
    assert "maxk.maxk_forward.default" in targets
    assert "maxk.spgemm_forward.default" in targets


def test_autograd_reaches_the_registered_derivatives():
    # fake CPU tensors: the autograd engine needs a real device for cuda ones, the fake
    # kernels only shapes
    with FakeTensorMode():
        ptr = torch.empty(41, dtype=torch.int32, device="cpu")
        idx = torch.empty(200, dtype=torch.int32, device="cpu")
        val = torch.empty(200, device="cpu")
        x = torch.empty(40, 32, device="cpu", requires_grad=True)
        y = _layer(ptr, idx, val, x, 8)
        assert y.requires_grad
        y.sum().backward()
        assert x.grad is not None and x.grad.shape == (40, 32)


# ------------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_opcheck_every_operator(gpu):
    n, d, k = 300, 64, 16
    ptr, idx, val = _graph(n, 3000, gpu)
    x = torch.randn(n, d, device=gpu, generator=torch.Generator(device=gpu).manual_seed(1))
    sp_data, sp_index = mk.maxk_forward(x, k, return_index=True)
    g = torch.randn(n, d, device=gpu, generator=torch.Generator(device=gpu).manual_seed(2))
    # the backward accumulates in float atomics: compiled and eager runs may sum in another order
    tol = dict(atol=1e-5, rtol=1e-5)
    torch.library.opcheck(torch.ops.maxk.maxk_forward.default, (x, k))
    torch.library.opcheck(torch.ops.maxk.maxk_backward.default, (sp_data, sp_index, d))
    torch.library.opcheck(torch.ops.maxk.spgemm_forward.default,
                          (ptr, idx, val, sp_data, sp_index, n, idx.numel(), k, d), **tol)
    torch.library.opcheck(torch.ops.maxk.spgemm_backward.default,
                          (ptr, idx, val, g, sp_index, n, idx.numel(), k, d), **tol)


@pytest.mark.gpu
def test_compiled_layer_step_matches_eager(gpu):
    n, d, k = 500, 128, 16
    ptr, idx, val = _graph(n, 6000, gpu, seed=7)
    x0 = torch.randn(n, d, device=gpu, generator=torch.Generator(device=gpu).manual_seed(4))
    w = torch.randn(d, d, device=gpu, generator=torch.Generator(device=gpu).manual_seed(5)) / d

    def step(x):
        return (_layer(ptr, idx, val, x, k) @ w).square().sum()

    xe = x0.clone().requires_grad_(True)
    le = step(xe)
    le.backward()
    xc = x0.clone().requires_grad_(True)
    lc = torch.compile(step, backend="aot_eager", fullgraph=True)(xc)
    lc.backward()
    torch.testing.assert_close(lc, le, atol=1e-4, rtol=1e-5)
    torch.testing.assert_close(xc.grad, xe.grad, atol=1e-5, rtol=1e-5)
    assert xe.grad.abs().sum() > 0
