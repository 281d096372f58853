"""Numerics of the hand-written HIP kernels vs plain PyTorch fp32 references.

All tests here need an MI355X (``-m gpu``); they run the native kernels only
(the loader raises if libmxkernels.so is missing — no silent fallback).
"""
import pytest
import torch

from mxk8s.ops import gemm_bf16_tn, vector_add, rmsnorm, swiglu, rope, rope_tables
from mxk8s.ops.fused import rmsnorm_ref, swiglu_ref, rope_ref

pytestmark = pytest.mark.gpu


def _rand(shape, dev, seed, scale=1.0):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    return ((torch.rand(shape, device=dev, generator=g) * 2 - 1) * scale)


@pytest.mark.parametrize("n", [1, 3, 50000, 1 << 20, (1 << 20) + 5])
def test_vector_add_f32_exact(cuda_device, n):
    a = _rand((n,), cuda_device, 1)
    b = _rand((n,), cuda_device, 2)
    c = vector_add(a, b)
    assert torch.equal(c.cpu(), a.cpu() + b.cpu())


def test_vector_add_bf16(cuda_device):
    n = (1 << 20) + 7
    a = _rand((n,), cuda_device, 3).bfloat16()
    b = _rand((n,), cuda_device, 4).bfloat16()
    c = vector_add(a, b)
    ref = (a.float() + b.float()).bfloat16()
    assert torch.equal(c, ref)


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 256), (1024, 1024, 1024),
                                   (2048, 4096, 512)])
def test_gemm_fast_path_vs_fp32(cuda_device, M, N, K):
    a = _rand((M, K), cuda_device, 5).bfloat16()
    bt = _rand((N, K), cuda_device, 6).bfloat16()
    c = gemm_bf16_tn(a, bt)
    ref = a.float() @ bt.float().t()
    err = (c.float() - ref).abs().max().item()
    # bf16 output rounding: |ref| <= K, relative 2^-8
    assert err <= ref.abs().max().item() * 2 ** -7 + 1e-3, err


def test_gemm_narrow_c_stride(cuda_device):
    """ldc % 8 != 0 takes the 8-byte-store schedule (no widened dwordx4 tail)."""
    M, N, K = 512, 512, 256
    a = _rand((M, K), cuda_device, 21).bfloat16()
    bt = _rand((N, K), cuda_device, 22).bfloat16()
    buf = torch.zeros((M, N + 4), device=cuda_device, dtype=torch.bfloat16)
    out = buf[:, :N]
    gemm_bf16_tn(a, bt, out)
    ref = a.float() @ bt.float().t()
    assert (out.float() - ref).abs().max().item() <= ref.abs().max().item() * 2 ** -7 + 1e-3
    assert torch.count_nonzero(buf[:, N:]) == 0   # nothing written past N


@pytest.mark.parametrize("M,N,K", [(4096, 4096, 256), (1024, 768, 512), (512, 512, 64),
                                   (512, 768, 128), (768, 512, 192), (512, 512, 320),
                                   (512, 256, 448), (256, 512, 832), (512, 512, 1216)])
def test_gemm_every_schedule_vs_fp32(cuda_device, M, N, K):
    """Every non-ablation schedule of the 256x256 kernel; 4096^2 puts the
    XCD super-block map (16x16 tiles) in play, 1024x768 its MAP-0 fallback;
    K = 64 .. 1216 gives 1-19 K-tiles, every remainder of the one-barrier
    schedule's 6-K-tile slot cycle (47: 3 A slots x 2 B slots)."""
    from mxk8s.ops import _lib
    L = _lib.lib()
    a = _rand((M, K), cuda_device, 23).bfloat16()
    bt = _rand((N, K), cuda_device, 24).bfloat16()
    ref = a.float() @ bt.float().t()
    tol = ref.abs().max().item() * 2 ** -7 + 1e-3
    built = [v for v in range(L.mxk_gemm_bf16_tn_num_variants())
             if L.mxk_gemm_bf16_tn_variant_built(v) and not L.mxk_gemm_bf16_tn_is_ablation(v)]
    assert 52 in built and 26 in built and 1 in built   # default, round-3 default, narrow-C fallback
    for v in built:
        c = torch.full((M, N), float("nan"), device=cuda_device, dtype=torch.bfloat16)
        st = L.mxk_gemm_bf16_tn_variant(a.data_ptr(), bt.data_ptr(), c.data_ptr(), M, N, K, K, K, N,
                                        v, _lib.stream_ptr(cuda_device))
        _lib.check(st, f"variant {v}")
        err = (c.float() - ref).abs().max().item()
        assert err <= tol, (v, err)


@pytest.mark.parametrize("M,N,K,variants", [(8192, 8192, 8192, (26, 6, 47, 52)),
                                            (16384, 16384, 512, (26, 52)),
                                            (16384, 6144, 4096, (26, 6, 52))])
def test_gemm_headline_shapes_full_output_vs_fp32(cuda_device, M, N, K, variants):
    """The long-K headline shape and the XCD super-block map at 64x64 tiles,
    the WHOLE output against an fp32 GEMM (tolerance 2^-7 max|ref|)."""
    from mxk8s.ops import _lib
    L = _lib.lib()
    a = _rand((M, K), cuda_device, 31).bfloat16()
    bt = _rand((N, K), cuda_device, 32).bfloat16()
    ref = a.float() @ bt.float().t()
    tol = ref.abs().max().item() * 2 ** -7
    for v in variants:
        c = torch.full((M, N), float("nan"), device=cuda_device, dtype=torch.bfloat16)
        st = L.mxk_gemm_bf16_tn_variant(a.data_ptr(), bt.data_ptr(), c.data_ptr(), M, N, K, K, K, N,
                                        v, _lib.stream_ptr(cuda_device))
        _lib.check(st, f"variant {v}")
        err = (c.float() - ref).abs().max().item()
        assert err <= tol, (v, err, tol)


@pytest.mark.parametrize("variant", [54, 55, 57])
@pytest.mark.parametrize("reserved", [0, 64])
@pytest.mark.parametrize("M,N,K", [(8192, 4096, 256), (4096, 8192, 1152), (8192, 8192, 2048)])
def test_gemm_staggered_rounds_vs_fp32(cuda_device, M, N, K, reserved, variant):
    """Schedules 54 / 55 (experiments library): half of each XCD's CUs start
    with half a tile (K-split tiles whose halves meet through uncached / plain
    memory and a flag).  Whole output against fp32, three launches back to
    back on one stream (the consumers reset the flags), also with the plan
    sized for 192 CUs."""
    from mxk8s.ops import _lib, gemm
    L = _lib.lib()
    if not L.mxk_gemm_bf16_tn_variant_built(variant):
        pytest.skip("experiments library only")
    T = (M // 256) * (N // 256)
    a = _rand((M, K), cuda_device, 41).bfloat16()
    bt = _rand((N, K), cuda_device, 42).bfloat16()
    ref = a.float() @ bt.float().t()
    tol = ref.abs().max().item() * 2 ** -7 + 1e-3
    try:
        gemm.set_reserved_cus(reserved)
        if variant == 57:
            cx = gemm.available_cus() // 8
            assert T % 8 == 0 and T // 8 >= 2 * cx, "shape too small for schedule 57"
        else:
            assert gemm.stagger_plan(T, K, gemm.available_cus()) > 0
        outs = []
        for _ in range(3):
            c = torch.full((M, N), float("nan"), device=cuda_device, dtype=torch.bfloat16)
            _lib.check(L.mxk_gemm_bf16_tn_variant(a.data_ptr(), bt.data_ptr(), c.data_ptr(), M, N, K,
                                                  K, K, N, variant, _lib.stream_ptr(cuda_device)),
                       f"v{variant}")
            outs.append(c)
        torch.cuda.synchronize()
    finally:
        gemm.set_reserved_cus(0)
    for c in outs:
        assert (c.float() - ref).abs().max().item() <= tol
        assert torch.equal(c, outs[0])


@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (17, 33, 65), (100, 300, 200), (255, 257, 63)])
def test_gemm_generic_path_vs_fp32(cuda_device, M, N, K):
    a = _rand((M, K), cuda_device, 7).bfloat16()
    bt = _rand((N, K), cuda_device, 8).bfloat16()
    c = gemm_bf16_tn(a, bt)
    ref = a.float() @ bt.float().t()
    err = (c.float() - ref).abs().max().item()
    assert err <= ref.abs().max().item() * 2 ** -7 + 1e-3, err


def test_gemm_identity_asymmetric(cuda_device):
    """A = I with an asymmetric B catches a transposed C write (guide §3)."""
    n = 512
    a = torch.eye(n, device=cuda_device, dtype=torch.bfloat16)
    idx = torch.arange(n, device=cuda_device, dtype=torch.float32)
    bt = ((idx[:, None] * 3 + idx[None, :] * 0.5) % 64).bfloat16()   # bt[j][k]
    c = gemm_bf16_tn(a, bt)   # c[i][j] = sum_k I[i][k] bt[j][k] = bt[j][i]
    assert torch.equal(c, bt.t().contiguous())


def test_gemm_exact_integers(cuda_device):
    M, N, K = 512, 512, 512
    g = torch.Generator(device=cuda_device)
    g.manual_seed(9)
    a = torch.randint(-2, 3, (M, K), device=cuda_device, generator=g).bfloat16()
    bt = torch.randint(-2, 3, (N, K), device=cuda_device, generator=g).bfloat16()
    c = gemm_bf16_tn(a, bt)
    ref = (a.double() @ bt.double().t())
    # |ref| <= 2048 < 2^8 * 8 -> integers up to 256 exact in bf16; compare in bf16
    assert torch.equal(c, ref.float().bfloat16())


def test_gemm_large_vs_hipblaslt(cuda_device):
    M = N = K = 4096
    a = _rand((M, K), cuda_device, 10).bfloat16()
    bt = _rand((N, K), cuda_device, 11).bfloat16()
    c = gemm_bf16_tn(a, bt).float()
    ref = torch.matmul(a, bt.t()).float()
    rel = ((c - ref).norm() / ref.norm()).item()
    assert rel <= 1e-2, rel


@pytest.mark.parametrize("rows,H", [(1, 4096), (7, 4096), (2048, 4096), (33, 2048), (5, 8192), (3, 128),
                                    (4096, 2048), (1024, 8192), (3000, 4096)])
def test_rmsnorm_fwd_bwd(cuda_device, rows, H):
    x = _rand((rows, H), cuda_device, 12, 3.0).bfloat16().requires_grad_()
    w = (1 + 0.1 * _rand((H,), cuda_device, 13)).bfloat16().requires_grad_()
    y = rmsnorm(x, w, 1e-5)
    assert (y.float() - rmsnorm_ref(x.detach(), w.detach(), 1e-5).float()).abs().max() < 3e-2
    dy = _rand((rows, H), cuda_device, 14).bfloat16()
    y.backward(dy)
    xr = x.detach().float().requires_grad_()
    wr = w.detach().float().requires_grad_()
    yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    yr.backward(dy.float())
    assert (x.grad.float() - xr.grad).abs().max() <= 2e-2 * xr.grad.abs().max() + 1e-3
    assert (w.grad.float() - wr.grad).abs().max() <= 2e-2 * wr.grad.abs().max() + 1e-3


@pytest.mark.parametrize("rows,F", [(1, 8), (2048, 14336), (3, 1000)])
def test_swiglu_fwd_bwd(cuda_device, rows, F):
    gu = _rand((rows, 2 * F), cuda_device, 15, 4.0).bfloat16().requires_grad_()
    h = swiglu(gu)
    assert (h.float() - swiglu_ref(gu.detach()).float()).abs().max() <= 0.05
    dh = _rand((rows, F), cuda_device, 16).bfloat16()
    h.backward(dh)
    gr = gu.detach().float().requires_grad_()
    g, u = gr.chunk(2, -1)
    (torch.nn.functional.silu(g) * u).backward(dh.float())
    assert (gu.grad.float() - gr.grad).abs().max() <= 2e-2 * gr.grad.abs().max() + 1e-2


@pytest.mark.parametrize("T,F,K", [(512, 768, 512), (2048, 1024, 4096), (1024, 512, 128)])
def test_swiglu_down_projection_fused_backward(cuda_device, T, F, K):
    """w2(swiglu(gu)) as one node: the SwiGLU backward runs in the epilogue of
    the input-gradient GEMM (mxk_gemm_bf16_dgrad_swiglu) - checked against an
    fp32 autograd reference of the plain composition, and the native kernel is
    checked to be the one that ran (no silent unfused fallback)."""
    from mxk8s.ops import _lib
    from mxk8s.ops.linear import SwiGLULinear, _dgrad_swiglu
    lin = SwiGLULinear(F, K).to(cuda_device).bfloat16()
    with torch.no_grad():
        lin.weight.copy_(_rand((K, F), cuda_device, 31, 0.05))
    gu = _rand((T, 2 * F), cuda_device, 32, 3.0).bfloat16().requires_grad_()
    y = lin(gu)
    dy = _rand((T, K), cuda_device, 33).bfloat16()
    y.backward(dy)
    gr = gu.detach().float().requires_grad_()
    wr = lin.weight.detach().float().requires_grad_()
    g, u = gr.chunk(2, -1)
    yr = (torch.nn.functional.silu(g) * u) @ wr.t()
    yr.backward(dy.float())
    assert (y.float() - yr).norm() / yr.norm() < 1e-2
    for got, ref, name in ((gu.grad, gr.grad, "dgu"), (lin.weight.grad, wr.grad, "dW")):
        rel = ((got.float() - ref).norm() / ref.norm()).item()
        assert rel < 1e-2, (name, rel)
    # every element (the epilogue's first row pass reads g / u from an LDS
    # prefetch, the other three from HBM)
    err = (gu.grad.float() - gr.grad).abs()
    assert err.max().item() <= 2 ** -6 * gr.grad.abs().max().item() + 1e-3, err.max().item()
    # the fused kernel itself accepts this shape
    dgu = torch.empty_like(gu)
    w = lin.weight.detach()
    st = _lib.lib().mxk_gemm_bf16_dgrad_swiglu(dy.data_ptr(), w.data_ptr(), gu.data_ptr(),
                                              dgu.data_ptr(), T, F, K, K, F,
                                              _lib.stream_ptr(cuda_device))
    assert st == 0
    assert torch.equal(dgu, _dgrad_swiglu(dy, w, gu.detach()))


@pytest.mark.parametrize("B,S,H,D", [(1, 2048, 32, 128), (2, 17, 8, 128), (1, 5, 3, 64)])
def test_rope_fwd_bwd(cuda_device, B, S, H, D):
    cos, sin = rope_tables(S, D, device=cuda_device)
    x = _rand((B, S, H, D), cuda_device, 17, 2.0).bfloat16().requires_grad_()
    y = rope(x, cos, sin)
    assert (y.float() - rope_ref(x.detach(), cos, sin).float()).abs().max() <= 3e-2
    dy = _rand((B, S, H, D), cuda_device, 18).bfloat16()
    y.backward(dy)
    xr = x.detach().float().requires_grad_()
    rope_ref(xr, cos, sin).backward(dy.float())
    assert (x.grad.float() - xr.grad).abs().max() <= 3e-2


@pytest.mark.parametrize("rows,H", [(7, 4096), (2048, 4096), (3, 256)])
def test_add_rmsnorm_fwd_bwd(cuda_device, rows, H):
    from mxk8s.ops.fused import add_rmsnorm
    x = _rand((rows, H), cuda_device, 21, 2.0).bfloat16().requires_grad_()
    d = _rand((rows, H), cuda_device, 22, 2.0).bfloat16().requires_grad_()
    w = (1 + 0.1 * _rand((H,), cuda_device, 23)).bfloat16().requires_grad_()
    h, y = add_rmsnorm(x, d, w, 1e-5)
    href = (x.detach() + d.detach())
    assert torch.equal(h, href)
    assert (y.float() - rmsnorm_ref(href, w.detach(), 1e-5).float()).abs().max() < 3e-2
    dh = _rand((rows, H), cuda_device, 24).bfloat16()
    dy = _rand((rows, H), cuda_device, 25).bfloat16()
    torch.autograd.backward([h, y], [dh, dy])
    xr = x.detach().float().requires_grad_()
    dr = d.detach().float().requires_grad_()
    wr = w.detach().float().requires_grad_()
    hr = xr + dr
    yr = hr * torch.rsqrt(hr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    torch.autograd.backward([hr, yr], [dh.float(), dy.float()])
    tol = 2e-2 * xr.grad.abs().max() + 1e-2
    assert (x.grad.float() - xr.grad).abs().max() <= tol
    assert (d.grad.float() - dr.grad).abs().max() <= tol
    assert (w.grad.float() - wr.grad).abs().max() <= 2e-2 * wr.grad.abs().max() + 1e-2


@pytest.mark.parametrize("variant", [0, 1, 2, 3])
@pytest.mark.parametrize("layout", ["tn", "nn", "nt_wgrad", "tt"])
@pytest.mark.parametrize("M,N,K", [(512, 768, 320), (4096, 4096, 192)])
def test_gemm_layouts_vs_fp32(cuda_device, layout, variant, M, N, K):
    """Layout-generic MFMA GEMM (K-major / N-major operands, tr_b16 reads);
    every schedule (auto, x, x2, x2 at hipBLASLt positions); 4096^2 puts the XCD
    super-block tile map in play."""
    from mxk8s.ops.gemm import gemm_bf16_ex
    g = torch.Generator(device=cuda_device).manual_seed(11)
    r = lambda *s: (torch.rand(*s, device=cuda_device, generator=g) * 2 - 1).bfloat16()  # noqa: E731
    if layout == "tn":
        a, b, ak, bk = r(M, K), r(N, K), True, True
        ref = a.float() @ b.float().t()
    elif layout == "nn":
        a, b, ak, bk = r(M, K), r(K, N), True, False
        ref = a.float() @ b.float()
    elif layout == "tt":
        a, b, ak, bk = r(K, M), r(N, K), False, True
        ref = a.float().t() @ b.float().t()
    else:
        a, b, ak, bk = r(K, M), r(K, N), False, False
        ref = a.float().t() @ b.float()
    out = torch.full((M, N), float("nan"), device=cuda_device, dtype=torch.bfloat16)
    assert gemm_bf16_ex(a, b, ak, bk, out, variant=variant)
    err = (out.float() - ref).abs().max().item()
    assert err <= 2 ** -7 * ref.abs().max().item() + 1e-3, err
    # shapes that do not tile fall back (nothing launched)
    assert not gemm_bf16_ex(a[:, :-64] if ak else a[:-64], b, ak, bk, out, variant=variant)


@pytest.mark.parametrize("layout", ["tn", "nn", "nt_wgrad", "tt"])
@pytest.mark.parametrize("M,N,K", [(4608, 4608, 1152), (8192, 8192, 2048), (1024, 768, 1216)])
def test_gemm_trickle_store_layouts_vs_fp32(cuda_device, layout, M, N, K):
    """Persistent trickle-store layout kernel (ex variant 4): 324 tiles on the
    CUs (some workgroups one tile, some two: the trickle phase runs for some,
    not others), 1024 tiles (four per CU, three trickle phases each) and a
    grid smaller than the chip; K at and above the 18-K-tile minimum.  The
    WHOLE output against fp32."""
    from mxk8s.ops import _lib
    from mxk8s.ops.gemm import gemm_bf16_ex
    if not _lib.lib().mxk_gemm_bf16_ex_variant_built(4):
        pytest.skip("x2t is an A/B record (experiments library only)")
    g = torch.Generator(device=cuda_device).manual_seed(13)
    r = lambda *s: (torch.rand(*s, device=cuda_device, generator=g) * 2 - 1).bfloat16()  # noqa: E731
    if layout == "tn":
        a, b, ak, bk = r(M, K), r(N, K), True, True
        ref = a.float() @ b.float().t()
    elif layout == "nn":
        a, b, ak, bk = r(M, K), r(K, N), True, False
        ref = a.float() @ b.float()
    elif layout == "tt":
        a, b, ak, bk = r(K, M), r(N, K), False, True
        ref = a.float().t() @ b.float().t()
    else:
        a, b, ak, bk = r(K, M), r(K, N), False, False
        ref = a.float().t() @ b.float()
    out = torch.full((M, N), float("nan"), device=cuda_device, dtype=torch.bfloat16)
    assert gemm_bf16_ex(a, b, ak, bk, out, variant=4)
    err = (out.float() - ref).abs().max().item()
    assert err <= 2 ** -7 * ref.abs().max().item() + 1e-3, err


@pytest.mark.parametrize("layout", ["nn", "nt_wgrad", "tt"])
@pytest.mark.parametrize("M,N,K", [(2048, 2048, 1024), (6144, 4096, 1024), (4096, 14336, 2048)])
def test_gemm_split_tail_vs_fp32(cuda_device, layout, M, N, K):
    """Split tail of the layout kernel: 64 tiles (all split, no whole-tile
    round), 384 and 896 tiles (the Llama-3-8B wqkv / w2 weight-gradient tile
    counts: one / three whole rounds + 128 tiles as K halves, fp32 partials
    summed by the fixup kernel).  The split path must actually run."""
    import ctypes

    from mxk8s.ops import _lib
    from mxk8s.ops.gemm import _split_workspace
    g = torch.Generator(device=cuda_device).manual_seed(5)
    r = lambda *s: (torch.rand(*s, device=cuda_device, generator=g) * 2 - 1).bfloat16()  # noqa: E731
    if layout == "nn":
        a, b, ak, bk = r(M, K), r(K, N), True, False
        ref = a.float() @ b.float()
    elif layout == "tt":
        a, b, ak, bk = r(K, M), r(N, K), False, True
        ref = a.float().t() @ b.float().t()
    else:
        a, b, ak, bk = r(K, M), r(K, N), False, False
        ref = a.float().t() @ b.float()
    out = torch.full((M, N), float("nan"), device=cuda_device, dtype=torch.bfloat16)
    ws = _split_workspace(cuda_device)
    cus = torch.cuda.get_device_properties(cuda_device).multi_processor_count
    tiles = (M // 256) * (N // 256)
    split = ctypes.c_int(-1)
    st = _lib.lib().mxk_gemm_bf16_ex_ws(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K,
                                        a.stride(0), b.stride(0), out.stride(0), int(ak), int(bk),
                                        ws.data_ptr(), ws.numel(), ctypes.byref(split),
                                        _lib.stream_ptr(cuda_device))
    _lib.check(st, "mxk_gemm_bf16_ex_ws")
    torch.cuda.synchronize()
    assert split.value == int(0 < tiles % cus <= cus // 2)
    err = (out.float() - ref).abs().max().item()
    assert err <= 2 ** -7 * ref.abs().max().item() + 1e-3, err


@pytest.mark.parametrize("T,V", [(4, 128256), (300, 1000), (7, 8)])
def test_fused_cross_entropy_vs_fp32(cuda_device, T, V):
    from mxk8s.ops.xent import cross_entropy
    g = torch.Generator(device=cuda_device).manual_seed(21)
    logits = (torch.randn(T, V, device=cuda_device, generator=g) * 3).bfloat16()
    labels = torch.randint(0, V, (T,), device=cuda_device, generator=g)
    if T > 4:
        labels[1] = -100          # ignore_index row: no loss, no gradient
    ref_in = logits.float().requires_grad_()
    ref = torch.nn.functional.cross_entropy(ref_in, labels, ignore_index=-100)
    ref.backward()
    x = logits.clone().requires_grad_()
    loss = cross_entropy(x, labels)
    assert abs(loss.item() - ref.item()) <= 1e-3 * max(1.0, abs(ref.item()))
    loss.backward()
    err = (x.grad.float() - ref_in.grad).abs().max().item()
    assert err <= 2 ** -8 * ref_in.grad.abs().max().item() + 1e-6, err


def test_qkv_rope_matches_split_rope(cuda_device):
    """Fused QKV split + RoPE (strided rope in/out, one d(qkv) buffer) equals
    split -> contiguous rope -> autograd concat, forward and backward."""
    from mxk8s.ops.fused import qkv_rope
    B, S, hq, hkv, hd = 2, 256, 8, 2, 128
    cos, sin = rope_tables(S, hd, device=cuda_device)
    qkv = _rand((B, S, (hq + 2 * hkv) * hd), cuda_device, 31, 2.0).bfloat16().requires_grad_()
    q, k, v = qkv_rope(qkv, cos, sin, hq, hkv, hd)
    ref_in = qkv.detach().clone().requires_grad_()
    rq, rk, rv = ref_in.split([hq * hd, hkv * hd, hkv * hd], dim=-1)
    rq = rope(rq.reshape(B, S, hq, hd).contiguous(), cos, sin)
    rk = rope(rk.reshape(B, S, hkv, hd).contiguous(), cos, sin)
    rv = rv.reshape(B, S, hkv, hd)
    for got, want in ((q, rq), (k, rk), (v, rv)):
        assert torch.equal(got, want)
    gq, gk, gv = (_rand(t.shape, cuda_device, 40 + i).bfloat16() for i, t in enumerate((q, k, v)))
    torch.autograd.backward((q, k, v), (gq, gk, gv))
    torch.autograd.backward((rq, rk, rv), (gq, gk, gv))
    assert torch.equal(qkv.grad, ref_in.grad)
    # ... and both against an independent fp32 PyTorch reference (rotate-half
    # RoPE in fp32; its gradient is the inverse rotation of the incoming grad)
    from mxk8s.ops.fused import rope_ref
    x32 = qkv.detach().float()
    fq, fk, fv = x32.split([hq * hd, hkv * hd, hkv * hd], dim=-1)
    want_q = rope_ref(fq.reshape(B, S, hq, hd), cos, sin)
    want_k = rope_ref(fk.reshape(B, S, hkv, hd), cos, sin)
    tol = 2 ** -7 * 4.0                        # bf16 output of |x| <= 2 rotated values
    assert (q.float() - want_q).abs().max().item() <= tol
    assert (k.float() - want_k).abs().max().item() <= tol
    assert torch.equal(v.float(), fv.reshape(B, S, hkv, hd))
    dq32 = rope_ref(gq.float(), cos, sin, sign=-1.0)
    dk32 = rope_ref(gk.float(), cos, sin, sign=-1.0)
    want_g = torch.cat([dq32.reshape(B, S, -1), dk32.reshape(B, S, -1), gv.float().reshape(B, S, -1)], -1)
    assert (qkv.grad.float() - want_g).abs().max().item() <= 2 ** -7 * 2.0


@pytest.mark.parametrize("a_kmajor,b_kmajor", [(1, 1), (1, 0), (0, 0)])
def test_gemm_exclusive_mode_vs_fp32(cuda_device, a_kmajor, b_kmajor):
    """Exclusive mode (each GEMM workgroup claims its CU's whole LDS through
    extra dynamic LDS) leaves the results unchanged: TN, dgrad and wgrad
    layouts and the fused SwiGLU up-projection."""
    from mxk8s.ops import gemm, linear
    M, N, K = 2048, 1024, 512
    a = _rand((M, K) if a_kmajor else (K, M), cuda_device, 51).bfloat16()
    b = _rand((N, K) if b_kmajor else (K, N), cuda_device, 52).bfloat16()
    ref = (a.float() if a_kmajor else a.float().t()) @ (b.float().t() if b_kmajor else b.float())
    try:
        gemm.set_exclusive(True)
        out = torch.empty((M, N), device=cuda_device, dtype=torch.bfloat16)
        assert gemm.gemm_bf16_ex(a, b, bool(a_kmajor), bool(b_kmajor), out)
        x = _rand((M, K), cuda_device, 53).bfloat16()
        w13 = _rand((2 * 512, K), cuda_device, 54).bfloat16()
        r = linear.w13_swiglu(x, w13)
        torch.cuda.synchronize()
    finally:
        gemm.set_exclusive(False)
    tol = ref.abs().max().item() * 2 ** -7 + 1e-3
    assert (out.float() - ref).abs().max().item() <= tol
    assert r is not None
    gu_ref = x.float() @ w13.float().t()
    assert (r[0].float() - gu_ref).abs().max().item() <= gu_ref.abs().max().item() * 2 ** -7 + 1e-3


@pytest.mark.parametrize("a_kmajor,b_kmajor", [(1, 0), (0, 0), (0, 1)])
def test_gemm_layouts_b_outer_order_vs_fp32(cuda_device, a_kmajor, b_kmajor):
    """The layout kernel's K-tile with the B fragment as the outer MFMA loop
    (mxk_gemm_x2_set_order(1), MXK_X2_ORDER=1; experiments library) against
    fp32, and the fused dgrad-SwiGLU GEMM under the same order against the
    default order."""
    from mxk8s.ops import _lib, gemm
    L = _lib.lib()
    if not L.mxk_gemm_bf16_tn_variant_built(54):
        pytest.skip("A/B record: experiments library only")
    M, N, K = 2048, 1024, 1088
    a = _rand((M, K) if a_kmajor else (K, M), cuda_device, 61).bfloat16()
    b = _rand((N, K) if b_kmajor else (K, N), cuda_device, 62).bfloat16()
    ref = (a.float() if a_kmajor else a.float().t()) @ (b.float().t() if b_kmajor else b.float())
    T, F, KD = 1024, 512, 1024
    dy = _rand((T, KD), cuda_device, 63).bfloat16()
    w2 = _rand((KD, F), cuda_device, 64, 0.05).bfloat16()
    gu = _rand((T, 2 * F), cuda_device, 65, 3.0).bfloat16()
    outs = []
    try:
        for order in (1, 0):
            L.mxk_gemm_x2_set_order(order)
            out = torch.empty((M, N), device=cuda_device, dtype=torch.bfloat16)
            assert gemm.gemm_bf16_ex(a, b, bool(a_kmajor), bool(b_kmajor), out)
            dgu = torch.empty_like(gu)
            _lib.check(L.mxk_gemm_bf16_dgrad_swiglu(dy.data_ptr(), w2.data_ptr(), gu.data_ptr(),
                                                    dgu.data_ptr(), T, F, KD, KD, F,
                                                    _lib.stream_ptr(cuda_device)), "dgrad_swiglu")
            torch.cuda.synchronize()
            outs.append((out, dgu))
    finally:
        L.mxk_gemm_x2_set_order(0)
    tol = ref.abs().max().item() * 2 ** -7 + 1e-3
    assert (outs[0][0].float() - ref).abs().max().item() <= tol
    d1, d0 = outs[0][1].float(), outs[1][1].float()
    assert (d1 - d0).abs().max().item() <= 2 ** -7 * d0.abs().max().item() + 1e-3


@pytest.mark.parametrize("reserved", [0, 64])
def test_dgrad_swiglu_staggered_vs_default(cuda_device, reserved):
    """Epilogue mode 8: the dgrad-SwiGLU GEMM with its rounds staggered by XCD
    group (first K halves hand fp32 partials to their second halves through
    uncached memory and flags; experiments library).  Against the default
    epilogue (mode 4) and an fp32 reference, launched three times back to back
    (flags reset)."""
    from mxk8s.ops import _lib, gemm
    L = _lib.lib()
    if not L.mxk_gemm_bf16_tn_variant_built(54):
        pytest.skip("A/B record: experiments library only")
    T, F, K = 4096, 8192, 1024
    dy = _rand((T, K), cuda_device, 71).bfloat16()
    w2 = _rand((K, F), cuda_device, 72, 0.05).bfloat16()
    gu = _rand((T, 2 * F), cuda_device, 73, 3.0).bfloat16()
    outs = {}
    try:
        gemm.set_reserved_cus(reserved)
        for mode in (8, 4):
            L.mxk_gemm_swiglu_set_epi(mode)
            runs = []
            for _ in range(3 if mode == 8 else 1):
                dgu = torch.full_like(gu, float("nan"))
                _lib.check(L.mxk_gemm_bf16_dgrad_swiglu(dy.data_ptr(), w2.data_ptr(), gu.data_ptr(),
                                                        dgu.data_ptr(), T, F, K, K, F,
                                                        _lib.stream_ptr(cuda_device)), f"mode {mode}")
                runs.append(dgu)
            torch.cuda.synchronize()
            outs[mode] = runs
    finally:
        L.mxk_gemm_swiglu_set_epi(4)
        gemm.set_reserved_cus(0)
    d = dy.float() @ w2.float()
    g, u = gu.float().chunk(2, -1)
    sg = torch.sigmoid(g)
    ref = torch.cat([d * u * sg * (1 + g * (1 - sg)), d * g * sg], -1)
    tol = 2 ** -6 * ref.abs().max().item() + 1e-3
    for dgu in outs[8]:
        assert not torch.isnan(dgu).any()
        assert (dgu.float() - ref).abs().max().item() <= tol
        assert torch.equal(dgu, outs[8][0])
    assert (outs[8][0].float() - outs[4][0].float()).abs().max().item() <= tol
