"""Fused softmax cross-entropy on bf16 logits (``native/kernels/xent.hip``).

``cross_entropy(logits [T, V] bf16, labels [T] int64)`` = mean over rows with
label >= 0 of ``logsumexp(logits) - logits[label]``, computed in fp32 inside
the kernel without an fp32 copy of the logits; the backward writes the bf16
gradient over the logits in place.  CPU / non-bf16 inputs use
``torch.nn.functional.cross_entropy`` (the reference the tests compare to).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib


class _XEnt(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        T, V = logits.shape
        loss_rows = torch.empty(T, dtype=torch.float32, device=logits.device)
        lse = torch.empty(T, dtype=torch.float32, device=logits.device)
        _lib.check(_lib.lib().mxk_xent_fwd(logits.data_ptr(), labels.data_ptr(),
                                           loss_rows.data_ptr(), lse.data_ptr(), T, V,
                                           logits.stride(0), _lib.stream_ptr(logits.device)),
                   "mxk_xent_fwd")
        count = (labels >= 0).sum().clamp_min(1).float()
        ctx.save_for_backward(logits, labels, lse, count)
        return loss_rows.sum() / count

    @staticmethod
    def backward(ctx, grad):
        logits, labels, lse, count = ctx.saved_tensors
        T, V = logits.shape
        g = (grad.float() / count).reshape(1).contiguous()
        # the logits are dead after the loss: their buffer becomes the gradient
        _lib.check(_lib.lib().mxk_xent_bwd(logits.data_ptr(), labels.data_ptr(), lse.data_ptr(),
                                           g.data_ptr(), T, V, logits.stride(0),
                                           _lib.stream_ptr(logits.device)), "mxk_xent_bwd")
        return logits, None


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    if logits.is_cuda and logits.dtype == torch.bfloat16 and logits.dim() == 2 and \
            logits.stride(1) == 1 and logits.shape[1] % 8 == 0 and logits.stride(0) % 8 == 0:
        return _XEnt.apply(logits, labels.reshape(-1).to(torch.int64).contiguous())
    return F.cross_entropy(logits.float(), labels.reshape(-1), ignore_index=-100)
