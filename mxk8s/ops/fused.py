"""Fused RMSNorm / SwiGLU / RoPE with autograd (``native/kernels/fused_ops.hip``).

Each op has a native HIP forward and backward for GPU tensors and a PyTorch
fp32 reference for CPU tensors (``*_ref``), which the numerics tests compare
the kernels against.
"""
from __future__ import annotations

import torch

from . import _lib

# ----------------------------------------------------------------------------
# references (fp32 math, output in the input dtype)
# ----------------------------------------------------------------------------


def rmsnorm_ref(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    rstd = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (xf * rstd * w.float()).to(x.dtype)


def swiglu_ref(gu: torch.Tensor) -> torch.Tensor:
    g, u = gu.float().chunk(2, dim=-1)
    return (torch.nn.functional.silu(g) * u).to(gu.dtype)


def rope_tables(seq_len: int, head_dim: int, theta: float = 500000.0,
                device=None) -> tuple[torch.Tensor, torch.Tensor]:
    """cos/sin tables [S, D/2] fp32 (host-precomputed; no device trig)."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    ang = torch.arange(seq_len, dtype=torch.float64)[:, None] * inv[None, :]
    return (ang.cos().float().contiguous().to(device), ang.sin().float().contiguous().to(device))


def rope_ref(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, sign: float = 1.0) -> torch.Tensor:
    """x: [B, S, H, D]; rotate-half pairing (i, i + D/2)."""
    S = x.shape[1]
    xf = x.float()
    half = x.shape[-1] // 2
    a, b = xf[..., :half], xf[..., half:]
    c = cos[:S].float()[None, :, None, :]
    s = sign * sin[:S].float()[None, :, None, :]
    return torch.cat([a * c - b * s, b * c + a * s], dim=-1).to(x.dtype)


# ----------------------------------------------------------------------------
# RMSNorm
# ----------------------------------------------------------------------------


# Norm weights marked ``_mxk_direct_grad`` (mxk8s.models.llama.RMSNorm) take
# the protocol of mxk8s.ops.linear: their gradient goes straight into
# ``weight.main_grad`` (the kernel writes it there on the first backward
# after zero_grad, later micro-batches add) and the DDP bucketer is told,
# instead of autograd's AccumulateGrad add into a zero-filled flat range.
def _direct_sink(w: torch.Tensor):
    if getattr(w, "_mxk_direct_grad", False) and getattr(w, "main_grad", None) is not None:
        return w.main_grad
    return None


def _deliver_dw(w: torch.Tensor, dw: torch.Tensor | None):
    """Finish a norm weight's gradient: None for autograd when it went to
    main_grad (``dw`` None: the kernel wrote it there), else ``dw``."""
    sink = _direct_sink(w)
    if sink is None:
        return dw
    if dw is not None:
        if w._mxk_grad_fresh:
            sink.copy_(dw)
        else:
            sink.add_(dw)
    w._mxk_grad_fresh = False
    ready = getattr(w, "_mxk_grad_ready", None)
    if ready is not None:
        ready()
    return None


def _dw_out(w: torch.Tensor) -> tuple[torch.Tensor, bool]:
    """(buffer the kernel writes dw into, whether that is main_grad)."""
    sink = _direct_sink(w)
    if sink is not None and w._mxk_grad_fresh and sink.dtype == w.dtype and sink.is_contiguous():
        return sink, True
    return torch.empty_like(w), False


class _RMSNormRef(torch.autograd.Function):
    """The fp32 reference (CPU / non-bf16) with the direct-gradient protocol
    for the weight."""

    @staticmethod
    def forward(ctx, x, w, eps):
        ctx.save_for_backward(x, w)
        ctx.eps = eps
        return rmsnorm_ref(x, w, eps)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        with torch.enable_grad():
            xx = x.detach().requires_grad_(ctx.needs_input_grad[0])
            ww = w.detach().requires_grad_(True)
            y = rmsnorm_ref(xx, ww, ctx.eps)
            ins = (xx, ww) if ctx.needs_input_grad[0] else (ww,)
            grads = torch.autograd.grad(y, ins, dy)
        dx = grads[0] if ctx.needs_input_grad[0] else None
        dw = grads[-1] if ctx.needs_input_grad[1] else None
        if dw is not None:
            dw = _deliver_dw(w, dw)
        return dx, dw, None



class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps):
        H = x.shape[-1]
        x2 = x.contiguous().view(-1, H)
        rows = x2.shape[0]
        y = torch.empty_like(x2)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        st = _lib.lib().mxk_rmsnorm_fwd(x2.data_ptr(), w.data_ptr(), y.data_ptr(),
                                        rstd.data_ptr(), rows, H, float(eps),
                                        _lib.stream_ptr(x.device))
        _lib.check(st, "mxk_rmsnorm_fwd")
        ctx.save_for_backward(x2, w, rstd)
        ctx.shape = x.shape
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w, rstd = ctx.saved_tensors
        rows, H = x2.shape
        dy2 = dy.contiguous().view(rows, H)
        dx = torch.empty_like(x2)
        dw, direct = _dw_out(w)
        L = _lib.lib()
        ws = torch.empty(L.mxk_rmsnorm_bwd_workspace(rows, H) // 4, dtype=torch.float32,
                         device=x2.device)
        st = L.mxk_rmsnorm_bwd(dy2.data_ptr(), x2.data_ptr(), w.data_ptr(), rstd.data_ptr(),
                               None, dx.data_ptr(), dw.data_ptr(), None, ws.data_ptr(), rows, H,
                               _lib.stream_ptr(x2.device))
        _lib.check(st, "mxk_rmsnorm_bwd")
        return dx.view(ctx.shape), _deliver_dw(w, None if direct else dw), None


class _AddRMSNorm(torch.autograd.Function):
    """h = x + delta ; y = rmsnorm(h) * w  ->  (h, y).  Backward fuses the
    residual gradient into the norm's input gradient: dx = ddelta =
    dh + rmsnorm_bwd(dy)."""

    @staticmethod
    def forward(ctx, x, delta, w, eps):
        H = x.shape[-1]
        x2 = x.contiguous().view(-1, H)
        d2 = delta.contiguous().view(-1, H)
        rows = x2.shape[0]
        h = torch.empty_like(x2)
        y = torch.empty_like(x2)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        st = _lib.lib().mxk_add_rmsnorm_fwd(x2.data_ptr(), d2.data_ptr(), w.data_ptr(), h.data_ptr(),
                                            y.data_ptr(), rstd.data_ptr(), rows, H, float(eps),
                                            _lib.stream_ptr(x.device))
        _lib.check(st, "mxk_add_rmsnorm_fwd")
        ctx.save_for_backward(h, w, rstd)
        ctx.shape = x.shape
        return h.view(x.shape), y.view(x.shape)

    @staticmethod
    def backward(ctx, dh, dy):
        h, w, rstd = ctx.saved_tensors
        rows, H = h.shape
        L = _lib.lib()
        dw, direct = _dw_out(w)
        if dy is None:
            dy = torch.zeros_like(h)
        dy2 = dy.contiguous().view(rows, H)
        dres = None if dh is None else dh.contiguous().view(rows, H)
        dx = torch.empty_like(h)
        ws = torch.empty(L.mxk_rmsnorm_bwd_workspace(rows, H) // 4, dtype=torch.float32,
                         device=h.device)
        st = L.mxk_rmsnorm_bwd(dy2.data_ptr(), h.data_ptr(), w.data_ptr(), rstd.data_ptr(),
                               None if dres is None else dres.data_ptr(), dx.data_ptr(),
                               dw.data_ptr(), None, ws.data_ptr(), rows, H,
                               _lib.stream_ptr(h.device))
        _lib.check(st, "mxk_rmsnorm_bwd")
        dx = dx.view(ctx.shape)
        return dx, dx, _deliver_dw(w, None if direct else dw), None


def add_rmsnorm(x: torch.Tensor, delta: torch.Tensor, w: torch.Tensor,
                eps: float = 1e-5) -> tuple[torch.Tensor, torch.Tensor]:
    """Fused pre-norm residual step: returns (h, rmsnorm(h) * w) with h = x + delta."""
    if x.device.type == "cpu" or x.dtype != torch.bfloat16:
        h = x + delta
        return h, rmsnorm(h, w, eps)
    return _AddRMSNorm.apply(x, delta, w, eps)


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    if x.device.type == "cpu" or x.dtype != torch.bfloat16:
        if getattr(w, "_mxk_direct_grad", False) and torch.is_grad_enabled():
            return _RMSNormRef.apply(x, w, eps)
        return rmsnorm_ref(x, w, eps)
    return _RMSNorm.apply(x, w, eps)


# ----------------------------------------------------------------------------
# SwiGLU over a fused [.., 2F] gate|up tensor
# ----------------------------------------------------------------------------


class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        F2 = gu.shape[-1]
        F = F2 // 2
        g2 = gu.contiguous().view(-1, F2)
        rows = g2.shape[0]
        h = torch.empty((rows, F), dtype=gu.dtype, device=gu.device)
        st = _lib.lib().mxk_swiglu_fwd(g2.data_ptr(), h.data_ptr(), rows, F,
                                       _lib.stream_ptr(gu.device))
        _lib.check(st, "mxk_swiglu_fwd")
        ctx.save_for_backward(g2)
        ctx.shape = gu.shape
        return h.view(*gu.shape[:-1], F)

    @staticmethod
    def backward(ctx, dh):
        (g2,) = ctx.saved_tensors
        rows, F2 = g2.shape
        dgu = torch.empty_like(g2)
        dh2 = dh.contiguous().view(rows, F2 // 2)
        st = _lib.lib().mxk_swiglu_bwd(g2.data_ptr(), dh2.data_ptr(), dgu.data_ptr(), rows,
                                       F2 // 2, _lib.stream_ptr(g2.device))
        _lib.check(st, "mxk_swiglu_bwd")
        return dgu.view(ctx.shape)


def swiglu_fwd(gu: torch.Tensor) -> torch.Tensor:
    """silu(g) * u of gu = [g | u] (bf16, GPU), no autograd node."""
    F = gu.shape[-1] // 2
    g2 = gu.contiguous().view(-1, 2 * F)
    h = torch.empty((g2.shape[0], F), dtype=gu.dtype, device=gu.device)
    _lib.check(_lib.lib().mxk_swiglu_fwd(g2.data_ptr(), h.data_ptr(), g2.shape[0], F,
                                         _lib.stream_ptr(gu.device)), "mxk_swiglu_fwd")
    return h.view(*gu.shape[:-1], F)


def swiglu_bwd(gu: torch.Tensor, dh: torch.Tensor) -> torch.Tensor:
    """d[g | u] from gu = [g | u] and dh = d(silu(g) * u) (bf16, GPU)."""
    F = gu.shape[-1] // 2
    g2 = gu.contiguous().view(-1, 2 * F)
    dh2 = dh.contiguous().view(-1, F)
    dgu = torch.empty_like(g2)
    _lib.check(_lib.lib().mxk_swiglu_bwd(g2.data_ptr(), dh2.data_ptr(), dgu.data_ptr(),
                                         g2.shape[0], F, _lib.stream_ptr(gu.device)),
               "mxk_swiglu_bwd")
    return dgu.view(gu.shape)


def swiglu(gu: torch.Tensor) -> torch.Tensor:
    if gu.device.type == "cpu" or gu.dtype != torch.bfloat16:
        g, u = gu.chunk(2, dim=-1)
        return torch.nn.functional.silu(g) * u
    return _SwiGLU.apply(gu)


# ----------------------------------------------------------------------------
# RoPE on [B, S, H, D]
# ----------------------------------------------------------------------------


def _rope_launch(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, sign: float,
                 out: torch.Tensor | None = None) -> torch.Tensor:
    """RoPE of x [B, S, H, D] into ``out`` (fresh contiguous by default).  x and
    out may be token-strided views ([B, S, H, D] with unit head/dim strides),
    e.g. slices of the fused QKV projection or of its gradient buffer."""
    B, S, H, D = x.shape
    if not (x.stride(3) == 1 and x.stride(2) == D and x.stride(0) == S * x.stride(1)):
        x = x.contiguous()
    y = torch.empty((B, S, H, D), dtype=x.dtype, device=x.device) if out is None else out
    assert y.stride(3) == 1 and y.stride(2) == D and y.stride(0) == S * y.stride(1)
    st = _lib.lib().mxk_rope_strided(x.data_ptr(), y.data_ptr(), cos.data_ptr(), sin.data_ptr(),
                                     B * S, H, D, S, float(sign), x.stride(1), y.stride(1),
                                     _lib.stream_ptr(x.device))
    _lib.check(st, "mxk_rope")
    return y


class _RoPE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cos, sin):
        ctx.save_for_backward(cos, sin)
        return _rope_launch(x, cos, sin, 1.0)

    @staticmethod
    def backward(ctx, dy):
        cos, sin = ctx.saved_tensors
        return _rope_launch(dy, cos, sin, -1.0), None, None


class _QKVRoPE(torch.autograd.Function):
    """Split of the fused QKV projection output + RoPE of q and k in one node:
    q and k are rotated straight out of their qkv slices (no contiguous
    copies), and the backward writes d(qkv) slice by slice into one buffer
    (RoPE-backward output strided into it) instead of autograd's split
    backward concatenating dq, dk and dv."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, hq: int, hkv: int, hd: int):
        B, S, _ = qkv.shape
        q = qkv[..., :hq * hd].view(B, S, hq, hd)
        k = qkv[..., hq * hd:(hq + hkv) * hd].view(B, S, hkv, hd)
        v = qkv[..., (hq + hkv) * hd:].view(B, S, hkv, hd)
        ctx.save_for_backward(cos, sin)
        ctx.dims = (hq, hkv, hd)
        return _rope_launch(q, cos, sin, 1.0), _rope_launch(k, cos, sin, 1.0), v

    @staticmethod
    def backward(ctx, dq, dk, dv):
        cos, sin = ctx.saved_tensors
        hq, hkv, hd = ctx.dims
        ref = dq if dq is not None else (dk if dk is not None else dv)
        B, S = ref.shape[:2]
        dqkv = torch.empty((B, S, (hq + 2 * hkv) * hd), dtype=ref.dtype, device=ref.device)
        for g, lo, h in ((dq, 0, hq), (dk, hq, hkv)):
            sl = dqkv[..., lo * hd:(lo + h) * hd].view(B, S, h, hd)
            if g is None:
                sl.zero_()
            else:
                _rope_launch(g, cos, sin, -1.0, out=sl)
        vs = dqkv[..., (hq + hkv) * hd:].view(B, S, hkv, hd)
        if dv is None:
            vs.zero_()
        else:
            vs.copy_(dv)
        return dqkv, None, None, None, None, None


def qkv_rope(qkv: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, hq: int, hkv: int,
             hd: int):
    """(q, k, v) of a fused projection output qkv [B, S, (hq + 2 hkv) hd], with
    rotary embedding applied to q and k; v is a view of qkv."""
    B, S, _ = qkv.shape
    if qkv.device.type == "cpu" or qkv.dtype != torch.bfloat16:
        q, k, v = qkv.split([hq * hd, hkv * hd, hkv * hd], dim=-1)
        return (rope_ref(q.reshape(B, S, hq, hd), cos, sin),
                rope_ref(k.reshape(B, S, hkv, hd), cos, sin), v.reshape(B, S, hkv, hd))
    return _QKVRoPE.apply(qkv, cos[:S].contiguous(), sin[:S].contiguous(), hq, hkv, hd)


def rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """Apply rotary embedding to x [B, S, H, D] with tables [>=S, D/2]."""
    if x.device.type == "cpu" or x.dtype != torch.bfloat16:
        return rope_ref(x, cos, sin)
    S = x.shape[1]
    cos_s = cos[:S].contiguous()
    sin_s = sin[:S].contiguous()
    return _RoPE.apply(x, cos_s, sin_s)


__all__ = ["rmsnorm", "add_rmsnorm", "swiglu", "rope", "qkv_rope", "rope_tables", "rmsnorm_ref",
           "swiglu_ref", "rope_ref"]
