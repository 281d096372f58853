"""HIP vector add (``native/kernels/vector_add.hip``): the smoke-test payload."""
from __future__ import annotations

import torch

from . import _lib


def vector_add(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    if a.shape != b.shape or a.dtype != b.dtype:
        raise ValueError("a and b must have the same shape and dtype")
    if a.dtype not in (torch.float32, torch.bfloat16):
        raise TypeError(f"unsupported dtype {a.dtype}")
    if not (a.is_contiguous() and b.is_contiguous()):
        raise ValueError("inputs must be contiguous")
    if out is None:
        out = torch.empty_like(a)
    if a.device.type == "cpu":
        out.copy_((a.float() + b.float()).to(a.dtype))
        return out
    L = _lib.lib()
    fn = L.mxk_vector_add_f32 if a.dtype == torch.float32 else L.mxk_vector_add_bf16
    st = fn(a.data_ptr(), b.data_ptr(), out.data_ptr(), a.numel(), _lib.stream_ptr(a.device))
    _lib.check(st, "mxk_vector_add")
    return out
