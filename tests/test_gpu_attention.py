"""GPU numerics of the hand-written flash attention (native/kernels/attention.hip)
against the fp32 PyTorch reference."""
import math

import pytest
import torch

from mxk8s.ops import attention as A

pytestmark = pytest.mark.gpu


def _qkv(B, S, Hq, Hkv, dev, seed=0, fused=False):
    g = torch.Generator(device=dev).manual_seed(seed)
    D = 128
    if fused:   # q/k/v as views of one fused projection output (Llama layout)
        qkv = torch.randn(B, S, (Hq + 2 * Hkv) * D, device=dev, generator=g).bfloat16()
        q, k, v = qkv.split([Hq * D, Hkv * D, Hkv * D], dim=-1)
        return q.view(B, S, Hq, D), k.view(B, S, Hkv, D), v.view(B, S, Hkv, D)
    mk = lambda h: torch.randn(B, S, h, D, device=dev, generator=g).bfloat16()  # noqa: E731
    return mk(Hq), mk(Hkv), mk(Hkv)


@pytest.mark.parametrize("B,S,Hq,Hkv,causal,fused", [
    (1, 128, 2, 1, True, False),
    (2, 256, 4, 2, True, False),
    (1, 512, 8, 2, True, True),
    (1, 384, 4, 4, False, False),
    (1, 256, 4, 1, False, True),
    (1, 2048, 32, 8, True, True),     # the Llama-3-8B step's attention shape (B = 1)
    (1, 1024, 4, 2, False, False),    # 16 tiles: every K / V ring slot reused
])
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6, 9, 10])
def test_attn_fwd_matches_reference(cuda_device, B, S, Hq, Hkv, causal, fused, variant):
    from mxk8s.ops import _lib
    if not _lib.lib().mxk_attn_fwd_variant_built(variant):
        pytest.skip(f"forward variant {variant} is an A/B record (experiments library only)")
    q, k, v = _qkv(B, S, Hq, Hkv, cuda_device, fused=fused)
    assert A.supported(q, k, v)
    o, lse = A.attn_fwd(q, k, v, causal=causal, variant=variant)
    ref = A.attention_ref(q, k, v, causal=causal)
    err = (o.float() - ref.float()).abs().max().item()
    assert err < 2e-2, err
    # LSE of the scaled scores, fp32 reference
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2).repeat_interleave(Hq // Hkv, dim=1)
    s = qf @ kf.transpose(-1, -2) / math.sqrt(128)
    if causal:
        s = s.masked_fill(torch.ones(S, S, dtype=torch.bool, device=cuda_device).triu(1), float("-inf"))
    assert torch.allclose(lse, torch.logsumexp(s, dim=-1), atol=1e-3, rtol=1e-4)


@pytest.mark.parametrize("B,S,Hq,Hkv,causal,fused", [
    (1, 128, 2, 1, True, False),
    (2, 256, 4, 2, True, True),
    (1, 512, 8, 2, True, False),
    (1, 256, 4, 4, False, False),
    (1, 2048, 32, 8, True, True),     # the Llama-3-8B step's attention shape (B = 1)
])
def test_attn_bwd_matches_reference(cuda_device, B, S, Hq, Hkv, causal, fused):
    q, k, v = _qkv(B, S, Hq, Hkv, cuda_device, seed=1, fused=fused)
    g = torch.Generator(device=cuda_device).manual_seed(7)
    dout = torch.randn(B, S, Hq, 128, device=cuda_device, generator=g).bfloat16()
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    ref = A.attention_ref(qr, kr, vr, causal=causal)
    ref.backward(dout.float())
    qh, kh, vh = (t.detach().clone().requires_grad_() for t in (q, k, v))
    out = A.flash_attention(qh, kh, vh, causal=causal)
    out.backward(dout)
    for name, got, want in (("dq", qh.grad, qr.grad), ("dk", kh.grad, kr.grad),
                            ("dv", vh.grad, vr.grad)):
        err = (got.float() - want).abs().max().item()
        tol = 3e-2 * max(1.0, want.abs().max().item())
        assert err < tol, (name, err, tol)


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("B,S,Hq,Hkv,causal", [
    (1, 256, 8, 2, True),
    (2, 384, 4, 1, True),
    (1, 256, 4, 4, False),
    (1, 2048, 32, 8, True),
])
def test_attn_bwd_variants_into_strided_dkdv(cuda_device, B, S, Hq, Hkv, causal, variant):
    """Both dK/dV schedules (per-q-head partials + reduce, GQA-fused), writing
    dk/dv into slices of one fused [dq | dk | dv] buffer (token stride)."""
    q, k, v = _qkv(B, S, Hq, Hkv, cuda_device, seed=3, fused=True)
    o, lse = A.attn_fwd(q, k, v, causal=causal)
    g = torch.Generator(device=cuda_device).manual_seed(9)
    dout = torch.randn(B, S, Hq, 128, device=cuda_device, generator=g).bfloat16()
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    A.attention_ref(qr, kr, vr, causal=causal).backward(dout.float())
    fused = torch.full((B, S, (Hq + 2 * Hkv) * 128), float("nan"), device=cuda_device,
                       dtype=torch.bfloat16)
    dk = fused[..., Hq * 128:(Hq + Hkv) * 128].view(B, S, Hkv, 128)
    dv = fused[..., (Hq + Hkv) * 128:].view(B, S, Hkv, 128)
    dq, dk2, dv2 = A.attn_bwd(q, k, v, o, lse, dout, causal=causal, dk=dk, dv=dv, variant=variant)
    assert dk2.data_ptr() == dk.data_ptr() and dv2.data_ptr() == dv.data_ptr()
    assert torch.isnan(fused[..., :Hq * 128]).all()   # the dq slice is not touched
    for name, got, want in (("dq", dq, qr.grad), ("dk", dk, kr.grad), ("dv", dv, vr.grad)):
        err = (got.float() - want).abs().max().item()
        tol = 3e-2 * max(1.0, want.abs().max().item())
        assert err < tol, (name, variant, err, tol)
    if variant == 5:   # the delta folded into dQ: bit-identical to the separate pass (3)
        ref3 = A.attn_bwd(q, k, v, o, lse, dout, causal=causal, variant=3)
        ref5 = A.attn_bwd(q, k, v, o, lse, dout, causal=causal, variant=5)
        for a3, a5 in zip(ref3, ref5):
            assert (a3.float() - a5.float()).abs().max().item() <= 1e-2 * max(1.0, a3.float().abs().max().item())


@pytest.mark.parametrize("B,S,Hq,Hkv,causal", [
    (1, 256, 4, 4, False),     # one key block, no GQA
    (2, 512, 8, 2, True),      # two key blocks: a masked wave per diagonal slice
    (1, 1024, 8, 1, True),     # MQA: all 8 query heads swept by one workgroup
    (1, 768, 4, 2, False),     # three key blocks, full attention
    (1, 2048, 32, 8, True),    # the Llama-3-8B shape (B = 1)
])
def test_attn_bwd_dkdv256_v6(cuda_device, B, S, Hq, Hkv, causal):
    """Backward variant 6: the 256-key-per-workgroup dK/dV kernel
    (attention_bwd256.hip, dK^T / dV^T in the accumulator file, S / dP with
    the key on the lane, -LSE/scale and -delta as the initial accumulators)
    after the delta-folded dQ kernel.  dK / dV vs the fp32 reference into
    strided slices of a fused buffer; bit-identical across two runs (no
    atomics anywhere); dQ bit-identical to variant 5 (same kernel, only the
    row constants it stores differ)."""
    q, k, v = _qkv(B, S, Hq, Hkv, cuda_device, seed=11, fused=True)
    o, lse = A.attn_fwd(q, k, v, causal=causal)
    g = torch.Generator(device=cuda_device).manual_seed(13)
    dout = torch.randn(B, S, Hq, 128, device=cuda_device, generator=g).bfloat16()
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    A.attention_ref(qr, kr, vr, causal=causal).backward(dout.float())
    fused = torch.full((B, S, (Hq + 2 * Hkv) * 128), float("nan"), device=cuda_device,
                       dtype=torch.bfloat16)
    dk = fused[..., Hq * 128:(Hq + Hkv) * 128].view(B, S, Hkv, 128)
    dv = fused[..., (Hq + Hkv) * 128:].view(B, S, Hkv, 128)
    dq, _, _ = A.attn_bwd(q, k, v, o, lse, dout, causal=causal, dk=dk, dv=dv, variant=6)
    for name, got, want in (("dq", dq, qr.grad), ("dk", dk, kr.grad), ("dv", dv, vr.grad)):
        assert not torch.isnan(got).any(), name
        err = (got.float() - want).abs().max().item()
        tol = 3e-2 * max(1.0, want.abs().max().item())
        assert err < tol, (name, err, tol)
    again = A.attn_bwd(q, k, v, o, lse, dout, causal=causal, variant=6)
    assert torch.equal(again[0], dq) and torch.equal(again[1], dk) and torch.equal(again[2], dv)
    v5 = A.attn_bwd(q, k, v, o, lse, dout, causal=causal, variant=5)
    assert torch.equal(v5[0], dq)
    for a5, a6 in zip(v5[1:], (dk, dv)):       # same math, other summation order
        scale_ = max(1.0, a5.float().abs().max().item())
        assert (a5.float() - a6.float()).abs().max().item() <= 1e-2 * scale_


@pytest.mark.parametrize("bf16_atomics", [False, True])
@pytest.mark.parametrize("B,S,Hq,Hkv,causal", [
    (1, 256, 4, 4, False),
    (2, 512, 8, 2, True),
    (1, 1024, 8, 1, True),
    (1, 2048, 32, 8, True),
])
def test_attn_bwd_onepass_v7_v8(cuda_device, B, S, Hq, Hkv, causal, bf16_atomics):
    """One-pass backward (variants 7 / 8): the 256-key workgroups also
    compute dQ = dS K from an LDS image of their dS and add it with fp32
    (7, into a zeroed fp32 accumulator, then a convert pass) or packed-bf16
    (8, straight into the zeroed dq) atomics.  Every output vs the fp32
    reference; dK / dV close to variant 6 (same kernel body; the prep pass
    sums delta = rowsum(dO * O) in another order than variant 6's dQ kernel,
    so dK differs in the last bits); dQ close to variant 6's deterministic
    dQ (fp32: summation order only)."""
    variant = 8 if bf16_atomics else 7
    q, k, v = _qkv(B, S, Hq, Hkv, cuda_device, seed=17, fused=True)
    o, lse = A.attn_fwd(q, k, v, causal=causal)
    g = torch.Generator(device=cuda_device).manual_seed(19)
    dout = torch.randn(B, S, Hq, 128, device=cuda_device, generator=g).bfloat16()
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    A.attention_ref(qr, kr, vr, causal=causal).backward(dout.float())
    dq, dk, dv = A.attn_bwd(q, k, v, o, lse, dout, causal=causal, variant=variant)
    for name, got, want in (("dq", dq, qr.grad), ("dk", dk, kr.grad), ("dv", dv, vr.grad)):
        assert not torch.isnan(got).any(), name
        err = (got.float() - want).abs().max().item()
        tol = 3e-2 * max(1.0, want.abs().max().item())
        assert err < tol, (name, err, tol)
    d6 = A.attn_bwd(q, k, v, o, lse, dout, causal=causal, variant=6)
    for name, a6, got in (("dk", d6[1], dk), ("dv", d6[2], dv)):
        err = (a6.float() - got.float()).abs().max().item()
        assert err <= 1e-2 * max(1.0, a6.float().abs().max().item()), (name, err)
    scale_ = max(1.0, d6[0].float().abs().max().item())
    lim = (2e-2 if bf16_atomics else 1e-2) * scale_
    assert (d6[0].float() - dq.float()).abs().max().item() <= lim


@pytest.mark.parametrize("B,S,Hq,Hkv,causal,fused", [
    (1, 256, 4, 1, False, False),    # one quad, one row block per tile ring slot
    (2, 512, 8, 2, True, True),      # two quads, diagonal steps, strided q / dk / dv
    (1, 1024, 8, 1, True, False),    # MQA: two quads of one KV head
    (1, 768, 8, 2, False, True),     # three 256-key blocks, full attention
    (1, 2048, 32, 8, True, True),    # the Llama-3-8B shape (B = 1)
    (1, 512, 4, 2, True, False),     # group of 2: not a quad -> variant 6 runs
])
def test_attn_bwd_dq256_v9(cuda_device, B, S, Hq, Hkv, causal, fused):
    """Backward variant 9: dQ by workgroups of the 4 query heads of a GQA quad
    x 64 rows, one wave per SIMD (attention_dq256.hip: Q / dO resident as MFMA
    operands in the accumulator file beside dQ^T, K / V by LDS-DMA shared by
    the 4 heads, the delta pass folded in), then the 256-key dK / dV.  Every
    output vs the fp32 reference into strided slices of a fused buffer;
    bit-identical across two runs (no atomics); close to variant 6 (same
    math, other summation order of dQ)."""
    q, k, v = _qkv(B, S, Hq, Hkv, cuda_device, seed=23, fused=fused)
    o, lse = A.attn_fwd(q, k, v, causal=causal)
    g = torch.Generator(device=cuda_device).manual_seed(29)
    dout = torch.randn(B, S, Hq, 128, device=cuda_device, generator=g).bfloat16()
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    A.attention_ref(qr, kr, vr, causal=causal).backward(dout.float())
    buf = torch.full((B, S, (Hq + 2 * Hkv) * 128), float("nan"), device=cuda_device,
                     dtype=torch.bfloat16)
    dk = buf[..., Hq * 128:(Hq + Hkv) * 128].view(B, S, Hkv, 128)
    dv = buf[..., (Hq + Hkv) * 128:].view(B, S, Hkv, 128)
    dq, _, _ = A.attn_bwd(q, k, v, o, lse, dout, causal=causal, dk=dk, dv=dv, variant=9)
    for name, got, want in (("dq", dq, qr.grad), ("dk", dk, kr.grad), ("dv", dv, vr.grad)):
        assert not torch.isnan(got).any(), name
        err = (got.float() - want).abs().max().item()
        tol = 3e-2 * max(1.0, want.abs().max().item())
        assert err < tol, (name, err, tol)
    again = A.attn_bwd(q, k, v, o, lse, dout, causal=causal, variant=9)
    assert torch.equal(again[0], dq) and torch.equal(again[1], dk) and torch.equal(again[2], dv)
    d6 = A.attn_bwd(q, k, v, o, lse, dout, causal=causal, variant=6)
    for name, a6, got in (("dq", d6[0], dq), ("dk", d6[1], dk), ("dv", d6[2], dv)):
        err = (a6.float() - got.float()).abs().max().item()
        assert err <= 1e-2 * max(1.0, a6.float().abs().max().item()), (name, err)
    if (Hq // Hkv) % 4:
        assert torch.equal(d6[0], dq)     # the fallback is variant 6 itself



@pytest.mark.parametrize("B,S,Hq,Hkv,causal", [
    (1, 256, 8, 2, True),
    (2, 512, 8, 2, False),
    (1, 512, 16, 4, True),
    (1, 256, 8, 1, True),
])
def test_qkv_rope_attention_fused_backward(cuda_device, B, S, Hq, Hkv, causal, monkeypatch):
    """The fused projection's split + RoPE + attention node
    (A.qkv_rope_attention): the forward equals qkv_rope + flash_attention
    bit for bit; its backward (variant 9 with the RoPE backward fused into
    the dQ / dK stores, mxk_attn_bwd_rope) returns the same d(qkv) as the
    unfused chain bit for bit, and matches the fp32 reference; the fallback
    (another backward variant: attention into the slices, then the RoPE
    passes) too."""
    from mxk8s.ops.fused import qkv_rope, rope_ref, rope_tables
    hd = 128
    g = torch.Generator(device=cuda_device).manual_seed(41)
    qkv = (torch.randn(B, S, (Hq + 2 * Hkv) * hd, device=cuda_device, generator=g) * 2).bfloat16()
    dout = torch.randn(B, S, Hq, hd, device=cuda_device, generator=g).bfloat16()
    cos, sin = rope_tables(S + 64, hd, device=cuda_device)

    x1 = qkv.clone().requires_grad_()
    o1 = A.qkv_rope_attention(x1, cos, sin, Hq, Hkv, hd, causal=causal)
    assert o1 is not None
    o1.backward(dout)

    x2 = qkv.clone().requires_grad_()
    q, k, v = qkv_rope(x2, cos, sin, Hq, Hkv, hd)
    o2 = A.flash_attention(q, k, v, causal=causal)
    o2.backward(dout)
    assert torch.equal(o1, o2)
    assert torch.equal(x1.grad, x2.grad)

    xr = qkv.float().requires_grad_()
    qr, kr, vr = xr.split([Hq * hd, Hkv * hd, Hkv * hd], dim=-1)
    qr = rope_ref(qr.reshape(B, S, Hq, hd), cos, sin)
    kr = rope_ref(kr.reshape(B, S, Hkv, hd), cos, sin)
    A.attention_ref(qr, kr, vr.reshape(B, S, Hkv, hd), causal=causal).backward(dout.float())
    err = (x1.grad.float() - xr.grad).abs().max().item()
    tol = 3e-2 * max(1.0, xr.grad.abs().max().item())
    assert err < tol, (err, tol)

    # the fallback inside the node's backward (variant 6 + stand-alone RoPE)
    monkeypatch.setattr(A, "_BWD_VARIANT", 6)
    x3 = qkv.clone().requires_grad_()
    A.qkv_rope_attention(x3, cos, sin, Hq, Hkv, hd, causal=causal).backward(dout)
    err = (x3.grad.float() - xr.grad).abs().max().item()
    assert err < tol, ("fallback", err, tol)


@pytest.mark.parametrize("B,S,Hq,Hkv,causal", [
    (1, 256, 8, 2, True),
    (2, 512, 16, 4, True),
    (1, 512, 8, 1, False),
])
def test_proj_rope_attention_fused(cuda_device, B, S, Hq, Hkv, causal):
    """The QKV projection with the rotary embedding in its GEMM epilogue
    (mxk_gemm_bf16_rope), attention on strided views of its output, and the
    fused RoPE backward (A.proj_rope_attention): the output bit for bit that
    of the same GEMM (schedule 52, no split tail) + qkv_rope +
    flash_attention; dx / dW those of the same chain's d(qkv) through the
    input- and weight-gradient GEMMs; all close to the fp32 reference."""
    from mxk8s.ops.fused import qkv_rope, rope_ref, rope_tables
    from mxk8s.ops.gemm import gemm_bf16_tn
    from mxk8s.ops.linear import _dgrad, _weight_grad
    hd, dim = 128, 256
    g = torch.Generator(device=cuda_device).manual_seed(43)
    x = torch.randn(B, S, dim, device=cuda_device, generator=g).bfloat16()
    w = (torch.randn((Hq + 2 * Hkv) * hd, dim, device=cuda_device, generator=g) / 8).bfloat16()
    dout = torch.randn(B, S, Hq, hd, device=cuda_device, generator=g).bfloat16()
    cos, sin = rope_tables(S, hd, device=cuda_device)

    x1, w1 = x.clone().requires_grad_(), w.clone().requires_grad_()
    o1 = A.proj_rope_attention(x1, w1, cos, sin, Hq, Hkv, hd, causal=causal)
    assert o1 is not None
    o1.backward(dout)

    qkv = torch.empty(B * S, w.shape[0], device=cuda_device, dtype=torch.bfloat16)
    gemm_bf16_tn(x.reshape(-1, dim), w, qkv)
    qkv = qkv.view(B, S, -1).requires_grad_()
    q, k, v = qkv_rope(qkv, cos, sin, Hq, Hkv, hd)
    o2 = A.flash_attention(q, k, v, causal=causal)
    o2.backward(dout)
    assert torch.equal(o1, o2)
    dqkv = qkv.grad.view(B * S, -1)
    assert torch.equal(x1.grad, _dgrad(dqkv, w).view(B, S, dim))
    assert torch.equal(w1.grad, _weight_grad(w, dqkv, x.reshape(-1, dim)))

    xr, wr = x.float().requires_grad_(), w.float().requires_grad_()
    qkvr = xr @ wr.t()
    qr, kr, vr = qkvr.split([Hq * hd, Hkv * hd, Hkv * hd], dim=-1)
    qr = rope_ref(qr.reshape(B, S, Hq, hd), cos, sin)
    kr = rope_ref(kr.reshape(B, S, Hkv, hd), cos, sin)
    A.attention_ref(qr, kr, vr.reshape(B, S, Hkv, hd), causal=causal).backward(dout.float())
    for name, got, want in (("dx", x1.grad, xr.grad), ("dw", w1.grad, wr.grad)):
        err = (got.float() - want).abs().max().item()
        tol = 5e-2 * max(1.0, want.abs().max().item())
        assert err < tol, (name, err, tol)
