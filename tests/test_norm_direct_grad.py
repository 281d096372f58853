"""RMSNorm weights marked _mxk_direct_grad (mxk8s.models.llama.RMSNorm):
the weight gradient goes straight into main_grad (overwrite while fresh,
add afterwards) with the DDP readiness call; the CPU reference path."""
import torch

from mxk8s.ops.fused import add_rmsnorm, rmsnorm, rmsnorm_ref


def _ref_grads(x, w, g):
    xr = x.clone().requires_grad_()
    wr = w.detach().clone().requires_grad_()
    rmsnorm_ref(xr, wr, 1e-5).backward(g)
    return xr.grad, wr.grad


def test_direct_weight_gradient_overwrites_then_adds():
    torch.manual_seed(0)
    x, g = torch.randn(4, 8, 16), torch.randn(4, 8, 16)
    x2, g2 = torch.randn(4, 8, 16), torch.randn(4, 8, 16)
    w = torch.nn.Parameter(torch.rand(16) + 0.5)
    dx_ref, dw1 = _ref_grads(x, w, g)
    _, dw2 = _ref_grads(x2, w, g2)
    w._mxk_direct_grad = True
    w.main_grad = torch.full_like(w, 9.0)
    w._mxk_grad_fresh = True
    calls = []
    w._mxk_grad_ready = lambda: calls.append(1)
    xd = x.clone().requires_grad_()
    rmsnorm(xd, w, 1e-5).backward(g)
    assert torch.allclose(xd.grad, dx_ref)
    assert torch.equal(w.main_grad, dw1) and w.grad is None
    assert calls == [1] and not w._mxk_grad_fresh
    rmsnorm(x2, w, 1e-5).backward(g2)
    assert torch.allclose(w.main_grad, dw1 + dw2) and calls == [1, 1]


def test_add_rmsnorm_reference_path_delivers_too():
    torch.manual_seed(1)
    x, d, g = torch.randn(2, 3, 8), torch.randn(2, 3, 8), torch.randn(2, 3, 8)
    w = torch.nn.Parameter(torch.rand(8) + 0.5)
    _, dw = _ref_grads(x + d, w, g)
    w._mxk_direct_grad = True
    w.main_grad = torch.zeros_like(w)
    w._mxk_grad_fresh = True
    _, y = add_rmsnorm(x, d, w, 1e-5)
    y.backward(g)
    assert torch.allclose(w.main_grad, dw) and w.grad is None


def test_unmarked_weight_keeps_autograd_gradient():
    torch.manual_seed(2)
    x, g = torch.randn(4, 16), torch.randn(4, 16)
    w = torch.nn.Parameter(torch.rand(16) + 0.5)
    _, dw = _ref_grads(x, w, g)
    rmsnorm(x, w, 1e-5).backward(g)
    assert torch.allclose(w.grad, dw)
