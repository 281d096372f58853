"""Flash attention on the hand-written gfx950 kernels
(``native/kernels/attention.hip``).

``flash_attention(q, k, v, causal=True)`` takes q [B, S, Hq, 128] and k/v
[B, S, Hkv, 128] bf16 tensors whose last two dims are contiguous (token
strides are free, so q/k/v may be views of a fused QKV projection) and
returns o [B, S, Hq, 128] — the layout the output projection consumes, no
transposes.  GQA: Hq % Hkv == 0.  The forward also produces the per-row
log-sum-exp that the backward kernel uses to recompute P.

``attention_ref`` is the fp32 PyTorch reference the tests compare against.
"""
from __future__ import annotations

import math
import os

import torch

from . import _lib

HEAD_DIM = 128
BLOCK_Q = 128


def supported(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor) -> bool:
    """Shapes/layouts the HIP kernels handle (others use the reference path)."""
    if q.device.type != "cuda" or q.dtype != torch.bfloat16:
        return False
    B, S, Hq, D = q.shape
    if D != HEAD_DIM or S % BLOCK_Q or k.shape[2] == 0 or Hq % k.shape[2]:
        return False
    for t in (q, k, v):
        if t.stride(-1) != 1 or t.stride(-2) != D or t.stride(0) != S * t.stride(1) \
                or t.stride(1) % 8 or t.data_ptr() % 16:
            return False
    return True


def attention_ref(q, k, v, causal: bool = True, scale: float | None = None) -> torch.Tensor:
    """fp32 reference: q [B,S,Hq,D], k/v [B,S,Hkv,D] -> [B,S,Hq,D] (q.dtype)."""
    B, S, Hq, D = q.shape
    Hkv = k.shape[2]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2).repeat_interleave(Hq // Hkv, dim=1)
    vf = v.float().transpose(1, 2).repeat_interleave(Hq // Hkv, dim=1)
    s = qf @ kf.transpose(-1, -2) * scale
    if causal:
        mask = torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1)
        s = s.masked_fill(mask, float("-inf"))
    o = torch.softmax(s, dim=-1) @ vf
    return o.transpose(1, 2).to(q.dtype)


def attn_fwd(q, k, v, causal: bool = True, scale: float | None = None, variant: int = 4):
    """HIP forward: returns (o [B,S,Hq,D] bf16, lse [B,Hq,S] fp32).

    ``variant`` 4 (default): K/V by LDS-DMA, software-pipelined body (exp of
    one P chunk under the PV MFMAs of the previous one), lazy rescale (the
    row max is only moved when it grows by more than 2^8), loop unrolled by
    two so the LDS read addresses are loop invariants - 0.313 vs 0.339 ms for
    variant 2 per Llama-3-8B layer (profiles/r2_attention/); 3 is 4 without
    the unroll, 2 the plain DMA body, 1 the plain body unrolled, 0 stages K/V
    through registers (A/B runs)."""
    B, S, Hq, D = q.shape
    Hkv = k.shape[2]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    o = torch.empty((B, S, Hq, D), dtype=q.dtype, device=q.device)
    lse = torch.empty((B, Hq, S), dtype=torch.float32, device=q.device)
    st = _lib.lib().mxk_attn_fwd_variant(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                         lse.data_ptr(), B, S, Hq, Hkv, D, q.stride(1),
                                         k.stride(1), v.stride(1), float(scale), int(causal),
                                         int(variant), _lib.stream_ptr(q.device))
    _lib.check(st, "mxk_attn_fwd")
    return o, lse


_BWD_VARIANT = int(os.environ.get("MXK_ATTN_BWD_VARIANT", "9"))


def attn_bwd(q, k, v, o, lse, dout, causal: bool = True, scale: float | None = None,
             dk=None, dv=None, variant: int | None = None):
    """HIP backward: returns (dq [B,S,Hq,D], dk [B,S,Hkv,D], dv [B,S,Hkv,D]).

    ``dk``/``dv`` may be preallocated views (e.g. slices of a fused dQKV
    buffer) with a token stride; by default they are fresh contiguous tensors.
    ``variant`` 9 (default; Hq / Hkv a multiple of 4 and S % 256 == 0, else
    6): dQ by workgroups of the 4 query heads of a GQA quad x 64 rows, one
    wave per SIMD (attention_dq256.hip: Q / dO resident as MFMA operands in
    the accumulator file, K / V by LDS-DMA shared by the four heads, dO / O /
    Q staged through LDS, the delta pass folded in), then variant 6's
    256-key dK / dV: bit-identical to variant 6 and 1-3 % faster per
    Llama-3-8B layer at B 8 (1.02-1.04 vs 1.045-1.057 ms,
    profiles/r6_dq256/SUMMARY.md).
    6: variant 5's dQ kernel (it
    also writes the row constants -lse/scale and -delta), then dK / dV by the
    256-key workgroups of attention_bwd256.hip (one wave per SIMD, dK^T / dV^T
    in accumulators, S / dP of both key tiles from one read of each Q / dO
    fragment, a key tile's softmax and dK / dV pipelined into the next step):
    1.018 vs 1.044 ms for variant 5 per Llama-3-8B layer at B 8, deterministic
    (profiles/r5_attention/).  8: one pass, dQ added by packed-bf16 atomics
    from the 256-key workgroups (0.983 ms; dQ summed in bf16 in a
    nondeterministic order); 7: the same with fp32 atomics and a convert pass
    (1.139 ms).  5: variant 3 with the delta pass (dO . O per query
    row) folded into the dQ kernel, which then runs before dK/dV: no separate
    delta kernel, 1.042 vs 1.064 ms per Llama-3-8B layer at B 8
    (profiles/r4_final/attention_b8.log).  3: variant 2 with explicitly software-pipelined
    dK/dV and dQ bodies (LDS operands read a group ahead instead of one
    lgkmcnt(0) per MFMA), bit-identical to 2 and 15 % faster (1.070 vs 1.262
    ms per Llama-3-8B layer at B 8: profiles/r2_attention/); 2: dK/dV
    accumulated over the query-head group in one workgroup, bf16 out, K/V and
    Q/dO tiles by LDS-DMA (1.21 vs 1.31-1.36 ms, profiles/r1_attention/);
    1: the same with register-staged tiles; 0: per-query-head fp32 partials
    + GQA reduce."""
    B, S, Hq, D = q.shape
    Hkv = k.shape[2]
    variant = _BWD_VARIANT if variant is None else variant
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    dout = dout.contiguous()
    dq = torch.empty((B, S, Hq, D), dtype=q.dtype, device=q.device)
    if dk is None:
        dk = torch.empty((B, S, Hkv, D), dtype=k.dtype, device=k.device)
    if dv is None:
        dv = torch.empty((B, S, Hkv, D), dtype=v.dtype, device=v.device)
    L = _lib.lib()
    ws = torch.empty(L.mxk_attn_bwd_workspace_variant(B, S, Hq, int(variant)) // 4,
                     dtype=torch.float32, device=q.device)
    st = L.mxk_attn_bwd_variant(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                dout.data_ptr(), lse.data_ptr(), dq.data_ptr(), dk.data_ptr(),
                                dv.data_ptr(), ws.data_ptr(), B, S, Hq, Hkv, D, q.stride(1),
                                k.stride(1), v.stride(1), dk.stride(1), dv.stride(1),
                                float(scale), int(causal), int(variant),
                                _lib.stream_ptr(q.device))
    _lib.check(st, "mxk_attn_bwd")
    return dq, dk, dv


class _FlashAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        o, lse = attn_fwd(q, k, v, causal=causal, scale=scale)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, dout):
        q, k, v, o, lse = ctx.saved_tensors
        dq, dk, dv = attn_bwd(q, k, v, o, lse, dout, causal=ctx.causal, scale=ctx.scale)
        return dq, dk, dv, None, None


# The fused projection's split + RoPE + attention as one autograd node
# (MXK_FUSED_ROPE_BWD=0 turns it off): the forward rotates q / k out of
# their qkv slices (the stand-alone RoPE pass) and runs the flash forward;
# the backward writes d(qkv) of the UN-rotated projection straight into one
# buffer - the RoPE backward fused into the dQ / dK stores of variant 9
# (mxk_attn_bwd_rope), dV in place - instead of separate dq / dk / dv, two
# RoPE passes over them and a dV copy (~400 MB of HBM traffic per
# Llama-3-8B layer at micro-batch 8).
_FUSED_ROPE_BWD = os.environ.get("MXK_FUSED_ROPE_BWD", "1") != "0"


class _QKVRoPEAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, hq: int, hkv: int, hd: int, causal: bool, scale):
        from .fused import _rope_launch
        B, S, _ = qkv.shape
        q = _rope_launch(qkv[..., :hq * hd].view(B, S, hq, hd), cos, sin, 1.0)
        k = _rope_launch(qkv[..., hq * hd:(hq + hkv) * hd].view(B, S, hkv, hd), cos, sin, 1.0)
        v = qkv[..., (hq + hkv) * hd:].view(B, S, hkv, hd)
        o, lse = attn_fwd(q, k, v, causal=causal, scale=scale)
        ctx.save_for_backward(q, k, v, o, lse, cos, sin)
        ctx.causal, ctx.scale, ctx.dims = causal, scale, (hq, hkv, hd)
        return o

    @staticmethod
    def backward(ctx, dout):
        q, k, v, o, lse, cos, sin = ctx.saved_tensors
        dqkv = _rope_attn_backward(q, k, v, o, lse, cos, sin, dout, ctx.dims, ctx.causal, ctx.scale)
        return dqkv, None, None, None, None, None, None, None


def _rope_attn_backward(q, k, v, o, lse, cos, sin, dout, dims, causal, scale):
    """d(qkv) [B, S, (hq + 2 hkv) hd] of the un-rotated projection from the
    rotated q / k the forward attended with."""
    from .fused import _rope_launch
    hq, hkv, hd = dims
    B, S = q.shape[:2]
    scale = scale if scale is not None else 1.0 / math.sqrt(hd)
    dqkv = torch.empty((B, S, (hq + 2 * hkv) * hd), dtype=q.dtype, device=q.device)
    dq = dqkv[..., :hq * hd].view(B, S, hq, hd)
    dk = dqkv[..., hq * hd:(hq + hkv) * hd].view(B, S, hkv, hd)
    dv = dqkv[..., (hq + hkv) * hd:].view(B, S, hkv, hd)
    dout = dout.contiguous()
    if _BWD_VARIANT == 9:
        L = _lib.lib()
        ws = torch.empty(L.mxk_attn_bwd_workspace_variant(B, S, hq, 9) // 4,
                         dtype=torch.float32, device=q.device)
        st = L.mxk_attn_bwd_rope(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                 dout.data_ptr(), lse.data_ptr(), dq.data_ptr(), dk.data_ptr(),
                                 dv.data_ptr(), ws.data_ptr(), B, S, hq, hkv, hd, q.stride(1),
                                 k.stride(1), v.stride(1), dq.stride(1), dk.stride(1),
                                 dv.stride(1), cos.data_ptr(), sin.data_ptr(), float(scale),
                                 int(causal), _lib.stream_ptr(q.device))
        if st == 0:
            return dqkv
        if st != 1:     # 1 = hipErrorInvalidValue: a layout variant 9 does not take
            _lib.check(st, "mxk_attn_bwd_rope")
    # other variants: the backward into the slices, then the RoPE passes
    gq, _, _ = attn_bwd(q, k, v, o, lse, dout, causal=causal, scale=scale, dk=dk, dv=dv)
    _rope_launch(gq, cos, sin, -1.0, out=dq)
    _rope_launch(dk, cos, sin, -1.0, out=dk)     # in place: a thread reads both halves first
    return dqkv


class _ProjRoPEAttention(torch.autograd.Function):
    """x -> qkv = x W^T -> RoPE(q, k) -> flash attention -> o as one node:
    the projection GEMM applies the rotary embedding in its epilogue
    (mxk_gemm_bf16_rope: q / k leave the GEMM rotated, no stand-alone RoPE
    pass and no rotated copies), the attention runs on q / k / v as strided
    views of that one buffer, and the backward takes d(qkv) of the
    un-rotated projection from the fused attention backward into the
    projection's input- and weight-gradient GEMMs (the weight gradient
    straight into the flat gradient buffer, as Linear does)."""

    @staticmethod
    def forward(ctx, x, weight, cos, sin, hq: int, hkv: int, hd: int, causal: bool, scale):
        from .fused import _rope_launch
        from .linear import _fwd
        B, S, K = x.shape
        x2 = x.reshape(-1, K)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        N = weight.shape[0]
        qkv = torch.empty((B * S, N), dtype=x.dtype, device=x.device)
        st = _lib.lib().mxk_gemm_bf16_rope(x2.data_ptr(), weight.data_ptr(), qkv.data_ptr(),
                                           B * S, N, K, x2.stride(0), weight.stride(0),
                                           qkv.stride(0), cos.data_ptr(), sin.data_ptr(), S,
                                           (hq + hkv) * hd, _lib.stream_ptr(x.device))
        qkv = qkv.view(B, S, N)
        q = qkv[..., :hq * hd].view(B, S, hq, hd)
        k = qkv[..., hq * hd:(hq + hkv) * hd].view(B, S, hkv, hd)
        v = qkv[..., (hq + hkv) * hd:].view(B, S, hkv, hd)
        if st != 0:
            if st != 1:
                _lib.check(st, "mxk_gemm_bf16_rope")
            qkv.copy_(_fwd(x2, weight).view(B, S, N))
            _rope_launch(q, cos, sin, 1.0, out=q)      # in place
            _rope_launch(k, cos, sin, 1.0, out=k)
        o, lse = attn_fwd(q, k, v, causal=causal, scale=scale)
        ctx.save_for_backward(x2, weight, q, k, v, o, lse, cos, sin)
        ctx.causal, ctx.scale, ctx.dims, ctx.xshape = causal, scale, (hq, hkv, hd), x.shape
        return o

    @staticmethod
    def backward(ctx, dout):
        from .linear import _dgrad, _weight_grad
        x2, weight, q, k, v, o, lse, cos, sin = ctx.saved_tensors
        dqkv = _rope_attn_backward(q, k, v, o, lse, cos, sin, dout, ctx.dims, ctx.causal, ctx.scale)
        dqkv2 = dqkv.view(-1, dqkv.shape[-1])
        need_x, need_w = ctx.needs_input_grad[:2]
        dx = _dgrad(dqkv2, weight).view(ctx.xshape) if need_x else None
        dw = _weight_grad(weight, dqkv2, x2) if need_w else None
        return dx, dw, None, None, None, None, None, None, None


def proj_rope_attention(x: torch.Tensor, weight: torch.Tensor, cos: torch.Tensor,
                        sin: torch.Tensor, hq: int, hkv: int, hd: int, causal: bool = True,
                        scale: float | None = None):
    """o [B, S, hq, hd] = attention(RoPE(split(x W^T))) as one node (see
    _ProjRoPEAttention); None when the layout is not the fused path's."""
    if not (_FUSED_ROPE_BWD and _FUSED_ROPE_FWD and x.is_cuda and x.dtype == torch.bfloat16
            and weight.dtype == torch.bfloat16 and x.dim() == 3 and weight.is_contiguous()
            and weight.shape[0] == (hq + 2 * hkv) * hd and hd == HEAD_DIM and hkv > 0
            and hq % hkv == 0 and (hq // hkv) % 4 == 0 and x.shape[1] % 256 == 0
            and cos.shape[0] >= x.shape[1]):
        return None
    S = x.shape[1]
    return _ProjRoPEAttention.apply(x, weight, cos[:S].float().contiguous(),
                                    sin[:S].float().contiguous(), hq, hkv, hd, causal, scale)


# the rotary embedding in the fused QKV projection's GEMM epilogue
# (MXK_FUSED_ROPE_FWD=0: the GEMM, then the stand-alone RoPE pass)
_FUSED_ROPE_FWD = os.environ.get("MXK_FUSED_ROPE_FWD", "1") != "0"


def qkv_rope_attention(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, hq: int, hkv: int,
                       hd: int, causal: bool = True, scale: float | None = None):
    """Attention output o [B, S, hq, hd] of a fused projection qkv [B, S,
    (hq + 2 hkv) hd] with rotary embedding on q and k, as one autograd node
    whose backward returns d(qkv) from the fused kernels; None when the
    layout is not the fused path's (the caller then runs qkv_rope +
    flash_attention)."""
    if not (_FUSED_ROPE_BWD and qkv.is_cuda and qkv.dtype == torch.bfloat16 and qkv.dim() == 3
            and qkv.is_contiguous() and qkv.data_ptr() % 16 == 0 and hd == HEAD_DIM
            and hkv > 0 and hq % hkv == 0 and (hq // hkv) % 4 == 0
            and qkv.shape[-1] == (hq + 2 * hkv) * hd and qkv.shape[1] % 256 == 0
            and cos.shape[0] >= qkv.shape[1]):
        return None
    S = qkv.shape[1]
    return _QKVRoPEAttention.apply(qkv, cos[:S].float().contiguous(), sin[:S].float().contiguous(),
                                   hq, hkv, hd, causal, scale)


def flash_attention(q, k, v, causal: bool = True, scale: float | None = None) -> torch.Tensor:
    """Attention o [B,S,Hq,D] for q [B,S,Hq,D], k/v [B,S,Hkv,D] (GQA).

    Runs the HIP kernels for supported CUDA bf16 inputs (``supported``);
    CPU / other dtypes take the fp32 reference (used by the CPU tests)."""
    if supported(q, k, v):
        return _FlashAttention.apply(q, k, v, causal, scale)
    if q.device.type == "cuda":
        raise RuntimeError(f"flash_attention: unsupported shape/layout on GPU: q {tuple(q.shape)} "
                           f"strides {q.stride()} (need head_dim 128, S % 128 == 0)")
    return attention_ref(q, k, v, causal=causal, scale=scale)
