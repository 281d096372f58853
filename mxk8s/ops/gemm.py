"""bf16 MFMA GEMM op (``native/kernels/gemm_bf16.hip``).

``gemm_bf16_tn(a, bt)`` computes ``a @ bt.T`` with ``a`` [M, K] and ``bt``
[N, K] (the nn.Linear weight layout), fp32 accumulation, bf16 output.
GPU tensors always run the hand-written CDNA4 kernel (256x256 MFMA tile when
M, N are multiples of 256 and K of 64, a bounds-checked 64x64 MFMA kernel
otherwise); CPU tensors use an fp32 PyTorch reference.
"""
from __future__ import annotations

import torch

from . import _lib


def _check_operand(t: torch.Tensor, name: str) -> None:
    if t.dtype != torch.bfloat16:
        raise TypeError(f"{name} must be bfloat16, got {t.dtype}")
    if t.dim() != 2:
        raise ValueError(f"{name} must be 2-D, got shape {tuple(t.shape)}")
    if t.stride(1) != 1:
        raise ValueError(f"{name} must be K-contiguous (stride(1) == 1)")


def gemm_bf16_tn(a: torch.Tensor, bt: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    _check_operand(a, "a")
    _check_operand(bt, "bt")
    M, K = a.shape
    N, K2 = bt.shape
    if K != K2:
        raise ValueError(f"K mismatch: a is {tuple(a.shape)}, bt is {tuple(bt.shape)}")
    if a.device.type == "cpu":
        ref = (a.float() @ bt.float().t()).to(torch.bfloat16)
        if out is not None:
            out.copy_(ref)
            return out
        return ref
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    else:
        _check_operand(out, "out")
        if tuple(out.shape) != (M, N):
            raise ValueError(f"out must be [{M}, {N}]")
    L = _lib.lib()
    st = L.mxk_gemm_bf16_tn(a.data_ptr(), bt.data_ptr(), out.data_ptr(), M, N, K,
                            a.stride(0), bt.stride(0), out.stride(0),
                            _lib.stream_ptr(a.device))
    _lib.check(st, "mxk_gemm_bf16_tn")
    return out


def is_fast_shape(M: int, N: int, K: int) -> bool:
    return M % 256 == 0 and N % 256 == 0 and K % 64 == 0


def gemm_flops(M: int, N: int, K: int) -> float:
    return 2.0 * M * N * K
