"""Fused MLP forward (mxk_gemm_bf16_w13_swiglu: up-projection with SwiGLU in
the GEMM epilogue) and the TN split tail, against fp32 PyTorch references."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.mark.parametrize("sched", [0, 1, 2, 3])
@pytest.mark.parametrize("M,F,K", [(256, 128, 64), (512, 384, 256), (2048, 1792, 1024),
                                   (512, 256, 448), (16384, 14336, 4096)])
def test_w13_swiglu_vs_fp32(dev, M, F, K, sched):
    """The production K loop (0: three-barrier w4j) and the experiments
    library's A/B records (1: the one-barrier loop of TN schedule 52, whose
    6-K-tile slot cycle K = 448 leaves at a remainder; 2: non-temporal gu;
    3: the persistent form, several tiles per workgroup at the larger
    shapes)."""
    from mxk8s.ops import _lib
    from mxk8s.ops.linear import w13_swiglu
    if sched and not _lib.lib().mxk_gemm_bf16_tn_variant_built(54):
        pytest.skip("A/B record: experiments library only")
    g = torch.Generator(device=dev).manual_seed(M + F + K)
    x = (torch.randn((M, K), device=dev, generator=g) * 0.5).bfloat16()
    w = (torch.randn((2 * F, K), device=dev, generator=g) * K ** -0.5).bfloat16()
    try:
        _lib.lib().mxk_gemm_w13_set_sched(sched)
        r = w13_swiglu(x, w)
        torch.cuda.synchronize()
    finally:
        _lib.lib().mxk_gemm_w13_set_sched(0)
    assert r is not None, "fused kernel did not take the shape"
    gu, h = r
    ref = x.float() @ w.float().t()
    tol = 2 ** -7 * ref.abs().max().item() + 1e-3
    assert (gu.float() - ref).abs().max().item() <= tol
    href = torch.nn.functional.silu(ref[:, :F]) * ref[:, F:]
    assert (h.float() - href).abs().max().item() <= 2 ** -7 * href.abs().max().item() + 1e-3


def test_w13_swiglu_refuses_untileable(dev):
    from mxk8s.ops.linear import w13_swiglu
    x = torch.zeros((200, 64), device=dev, dtype=torch.bfloat16)
    w = torch.zeros((256, 64), device=dev, dtype=torch.bfloat16)
    assert w13_swiglu(x, w) is None


def test_fused_mlp_node_matches_unfused_autograd(dev):
    """forward + backward of the one-node MLP vs the two-node composition."""
    from mxk8s.ops.fused import swiglu
    from mxk8s.ops.linear import swiglu_mlp
    torch.manual_seed(0)
    M, D, F = 512, 256, 384
    x = (torch.randn(2, M // 2, D, device=dev) * 0.5).bfloat16().requires_grad_()
    w13 = (torch.randn(2 * F, D, device=dev) * D ** -0.5).bfloat16().requires_grad_()
    w2 = (torch.randn(D, F, device=dev) * F ** -0.5).bfloat16().requires_grad_()
    y = swiglu_mlp(x, w13, w2)
    dy = torch.randn_like(y)
    y.backward(dy)
    xr, w13r, w2r = (t.detach().float().requires_grad_() for t in (x, w13, w2))
    yr = swiglu(xr @ w13r.t()) @ w2r.t()
    yr.backward(dy.float())
    for got, ref in ((y, yr), (x.grad, xr.grad), (w13.grad, w13r.grad), (w2.grad, w2r.grad)):
        err = (got.float() - ref).abs().max().item()
        assert err <= 2 ** -6 * ref.abs().max().item() + 1e-2, err


@pytest.mark.parametrize("M,N,K", [(2048, 4096, 4096), (256 * 24, 256 * 16, 1024)])
def test_tn_split_tail_vs_fp32(dev, M, N, K):
    """Forward GEMMs whose last round of tiles is at most half full run the
    split tail (two K halves per tail tile + fixup)."""
    from mxk8s.ops.gemm import gemm_bf16_ex
    g = torch.Generator(device=dev).manual_seed(7)
    a = (torch.rand((M, K), device=dev, generator=g) * 2 - 1).bfloat16()
    b = (torch.rand((N, K), device=dev, generator=g) * 2 - 1).bfloat16()
    out = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    assert gemm_bf16_ex(a, b, True, True, out)
    ref = a.float() @ b.float().t()
    assert (out.float() - ref).abs().max().item() <= 2 ** -7 * ref.abs().max().item() + 1e-3
