"""Bias-free linear layer whose weight gradient is written straight into the
flat gradient buffer of :class:`~mxk8s.parallel.ddp.FlatParamSpace`.

With stock ``nn.Linear`` autograd produces dW in a fresh tensor and
``AccumulateGrad`` adds it into the (pre-zeroed) flat ``.grad`` view: for
Llama-3-8B that is a 16 GB memset plus a 48 GB read-read-write add pass per
step (~10 ms on MI355X).  Here the dW GEMM (the hand-written layout kernel) writes its output
directly into ``weight.main_grad`` — overwrite on the first backward after
``zero_grad`` (so no memset), ``addmm_`` accumulation on later micro-batches —
and then tells the DDP bucketer that the gradient is ready (the role the
post-accumulate-grad hook plays for other parameters).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from .gemm import gemm_bf16_ex

# dW = dy^T x has both operands token-major ("NT"): the hand-written
# layout-generic MFMA kernel beats hipBLASLt there (profiles/r1_gemm_layouts:
# +10-29 % on the Llama-3-8B wo/w13/w2 shapes); MXK_WGRAD=0 selects hipBLASLt.
_USE_MXK_WGRAD = os.environ.get("MXK_WGRAD", "1") != "0"
# dx = dy W has a K-major dy and an N-major W: the x2 schedule of the layout
# kernel runs it at 1390-1450 TF/s on the Llama-3-8B shapes (16k tokens)
# against hipBLASLt's 1350-1390 (profiles/r1_gemm_w4h/gemm_layouts_x2.log);
# MXK_DGRAD=0 selects hipBLASLt.
_USE_MXK_DGRAD = os.environ.get("MXK_DGRAD", "1") != "0"


# y = x W^T (both operands K-major) runs on the hand-written TN kernel (the
# validator's GEMM, gemm_bf16.hip) with the split tail when the last round of
# tiles is at most half full; no library GEMM in the training step.  Shapes
# that do not tile (M, N % 256, K % 64; tests, toy models) take the kernel's
# bounds-checked MFMA path; CPU tensors the PyTorch reference.
# MXK_FWD_LIB=1 (A/B measurements only, with MXK_FUSED_W13=0): the forward
# products on torch.matmul / hipBLASLt, the round-2 routing, so a same-box
# step A/B can price the hand-written forward path.
_FWD_LIB = os.environ.get("MXK_FWD_LIB", "0") == "1"


def _fwd(x: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    if _FWD_LIB or not x.is_cuda or x.dtype != torch.bfloat16 or weight.dtype != torch.bfloat16:
        return torch.matmul(x, weight.t())
    x2 = x.reshape(-1, x.shape[-1])
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    out = torch.empty((x2.shape[0], weight.shape[0]), device=x.device, dtype=x.dtype)
    w = weight if weight.is_contiguous() else weight.contiguous()
    if not gemm_bf16_ex(x2, w, True, True, out):
        from .gemm import gemm_bf16_tn
        gemm_bf16_tn(x2, w, out)          # bounds-checked MFMA kernel (any shape)
    return out.view(*x.shape[:-1], weight.shape[0])


def _wgrad_into(sink: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor) -> None:
    # no tail-heavy exception here: even without its split tail the 384-tile
    # wqkv wgrad (6144 x 4096, 1.5 rounds on 256 CUs) ran 1215 TF/s on the
    # layout kernel against hipBLASLt's 1150 (profiles/r1_gemm_m0/llama_*.log)
    if _USE_MXK_WGRAD and sink.is_cuda and dy2.is_contiguous() and x2.is_contiguous() and \
            gemm_bf16_ex(dy2, x2, False, False, sink):
        return
    torch.matmul(dy2.t(), x2, out=sink)


def _dgrad(dy: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    # tail-heavy outputs take the kernel's split tail (gemm_bf16_ex)
    if _USE_MXK_DGRAD and dy.is_cuda and dy.is_contiguous() and weight.is_contiguous():
        dy2 = dy.reshape(-1, dy.shape[-1])
        out = torch.empty((dy2.shape[0], weight.shape[1]), device=dy.device, dtype=dy.dtype)
        if gemm_bf16_ex(dy2, weight, True, False, out):
            return out.view(*dy.shape[:-1], weight.shape[1])
    return torch.matmul(dy, weight)


def _weight_grad(weight: torch.Tensor, dy: torch.Tensor, x: torch.Tensor):
    """dW = dy^T x: straight into weight.main_grad when the weight lives in a
    flat gradient buffer (then returns None), else returned."""
    x2 = x.reshape(-1, x.shape[-1])
    dy2 = dy.reshape(-1, dy.shape[-1])
    sink = getattr(weight, "main_grad", None)
    if sink is None:
        return torch.matmul(dy2.t(), x2)
    if weight._mxk_grad_fresh:
        _wgrad_into(sink, dy2, x2)
        weight._mxk_grad_fresh = False
    else:
        sink.addmm_(dy2.t(), x2)
    ready = getattr(weight, "_mxk_grad_ready", None)
    if ready is not None:
        ready()
    return None


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight):
        ctx.save_for_backward(x, weight)
        return _fwd(x, weight)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dx = _dgrad(dy, weight) if ctx.needs_input_grad[0] else None
        dw = _weight_grad(weight, dy, x) if ctx.needs_input_grad[1] else None
        return dx, dw


# y = swiglu(gu) W^T with the SwiGLU backward fused into the input-gradient
# GEMM's epilogue (mxk_gemm_bf16_dgrad_swiglu): d(act) = dy W never goes to
# HBM (0.94 GB less traffic per Llama-3-8B layer, no separate element-wise
# pass, d(act) kept in fp32).  Round 1 measured it step-neutral (the 8-B
# per-lane g/u accesses made the epilogue slow); with the LDS-staged epilogue
# (whole-line g/u accesses) the kernel runs 1.52 ms against 1.71 and the step
# gains 1.1 % (profiles/r2_split_tail/).  MXK_FUSED_SWIGLU=0 runs the
# unfused pair.
_USE_FUSED_SWIGLU = os.environ.get("MXK_FUSED_SWIGLU", "1") != "0"


def _dgrad_swiglu(dy: torch.Tensor, weight: torch.Tensor, gu: torch.Tensor) -> torch.Tensor:
    from . import _lib
    from .fused import swiglu_bwd
    F = weight.shape[1]
    dy2 = dy.reshape(-1, dy.shape[-1])
    gu2 = gu.reshape(-1, 2 * F)
    if _USE_FUSED_SWIGLU and dy2.is_contiguous() and gu2.is_contiguous() and weight.is_contiguous():
        dgu = torch.empty_like(gu2)
        st = _lib.lib().mxk_gemm_bf16_dgrad_swiglu(
            dy2.data_ptr(), weight.data_ptr(), gu2.data_ptr(), dgu.data_ptr(), dy2.shape[0], F,
            dy2.shape[1], dy2.stride(0), weight.stride(0), _lib.stream_ptr(dy.device))
        if st == 0:
            return dgu.view(gu.shape)
    return swiglu_bwd(gu, _dgrad(dy, weight))


class _SwiGLULinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu, weight):
        from .fused import swiglu_fwd
        h = swiglu_fwd(gu)
        ctx.save_for_backward(gu, h, weight)
        return _fwd(h, weight)

    @staticmethod
    def backward(ctx, dy):
        gu, h, weight = ctx.saved_tensors
        dgu = _dgrad_swiglu(dy, weight, gu) if ctx.needs_input_grad[0] else None
        dw = _weight_grad(weight, dy, h) if ctx.needs_input_grad[1] else None
        return dgu, dw


# gu = x W13^T and h = silu(g) * u in ONE launch (mxk_gemm_bf16_w13_swiglu:
# the activation runs in the GEMM's epilogue from the fp32 accumulators, the
# separate element-wise pass over gu disappears).  MXK_FUSED_W13=0 runs the
# GEMM and mxk_swiglu_fwd separately.
_USE_FUSED_W13 = os.environ.get("MXK_FUSED_W13", "1") != "0"


def w13_swiglu(x2: torch.Tensor, w13: torch.Tensor):
    """(gu, h) of the MLP up-projection, or None when the fused kernel does not
    take the shape (M % 256, F % 128, K % 64, aligned, bf16 GPU tensors)."""
    from . import _lib
    if not (_USE_FUSED_W13 and x2.is_cuda and x2.dtype == torch.bfloat16 and
            w13.dtype == torch.bfloat16 and x2.is_contiguous() and w13.is_contiguous()):
        return None
    M, K = x2.shape
    F = w13.shape[0] // 2
    gu = torch.empty((M, 2 * F), device=x2.device, dtype=x2.dtype)
    h = torch.empty((M, F), device=x2.device, dtype=x2.dtype)
    st = _lib.lib().mxk_gemm_bf16_w13_swiglu(x2.data_ptr(), w13.data_ptr(), gu.data_ptr(),
                                             h.data_ptr(), M, F, K, x2.stride(0), w13.stride(0),
                                             gu.stride(0), h.stride(0), _lib.stream_ptr(x2.device))
    if st == 1:      # hipErrorInvalidValue: shape / alignment not taken
        return None
    _lib.check(st, "mxk_gemm_bf16_w13_swiglu")
    return gu, h


class _SwiGLUMLPFn(torch.autograd.Function):
    """y = swiglu(x W13^T) W2^T as one autograd node: fused up-projection +
    activation forward, fused dgrad-SwiGLU backward; both weight gradients go
    straight into the flat gradient buffer (W2's first, as autograd would
    order the two nodes)."""

    @staticmethod
    def forward(ctx, x, w13, w2):
        from .fused import swiglu_fwd
        x2 = x.reshape(-1, x.shape[-1])
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        r = w13_swiglu(x2, w13)
        if r is None:
            gu = _fwd(x2, w13)
            h = swiglu_fwd(gu)
        else:
            gu, h = r
        ctx.save_for_backward(x2, gu, h, w13, w2)
        ctx.xshape = x.shape
        return _fwd(h, w2).view(*x.shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, gu, h, w13, w2 = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        need_x, need_w13, need_w2 = ctx.needs_input_grad
        dgu = _dgrad_swiglu(dy2, w2, gu) if (need_x or need_w13) else None
        dw2 = _weight_grad(w2, dy2, h) if need_w2 else None
        dx = _dgrad(dgu, w13).view(ctx.xshape) if need_x else None
        dw13 = _weight_grad(w13, dgu, x2) if need_w13 else None
        return dx, dw13, dw2


def swiglu_mlp(x: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor) -> torch.Tensor:
    return _SwiGLUMLPFn.apply(x, w13, w2)


class Linear(nn.Linear):
    """``nn.Linear(bias=False)`` with the direct-to-flat-buffer weight gradient."""

    def __init__(self, in_features: int, out_features: int, **kw):
        super().__init__(in_features, out_features, bias=False, **kw)
        self.weight._mxk_direct_grad = True

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return _LinearFn.apply(x, self.weight)


class SwiGLULinear(Linear):
    """Down projection applied to swiglu(gu), gu = [gate | up] of width
    2 * in_features: ``w2(swiglu(gu))`` as one node whose backward fuses the
    SwiGLU gradient into the input-gradient GEMM.  CPU / non-bf16 inputs take
    the plain composition."""

    def forward(self, gu: torch.Tensor) -> torch.Tensor:
        if gu.device.type == "cpu" or gu.dtype != torch.bfloat16:
            from .fused import swiglu
            return super().forward(swiglu(gu))
        return _SwiGLULinearFn.apply(gu, self.weight)
