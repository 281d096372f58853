"""Token embedding whose weight gradient goes straight into the flat
gradient buffer (the protocol of :mod:`mxk8s.ops.linear`).

With ``nn.Embedding`` autograd builds a dense [vocab, dim] gradient and
``AccumulateGrad`` adds it into the (pre-zeroed) flat ``.grad`` view: for
Llama-3-8B's 128,256 x 4,096 table that is a 1 GB memset in ``zero_grad``
plus a 1 GB read-read-write add per step.  Here the dense backward writes
``weight.main_grad`` itself (``embedding_dense_backward.out``: every row,
untouched rows zero) on the first backward after ``zero_grad`` and adds on
later micro-batches, then reports the gradient ready to the DDP bucketer.
The values are the ones autograd's path produces (the same dense backward;
0 + g = g).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


def _notify_grad(weight: torch.Tensor) -> None:
    ready = getattr(weight, "_mxk_grad_ready", None)
    if ready is not None:
        ready()


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, tokens, weight):
        ctx.save_for_backward(tokens)
        ctx.weight = weight
        return F.embedding(tokens, weight)

    @staticmethod
    def backward(ctx, dy):
        (tokens,) = ctx.saved_tensors
        w = ctx.weight
        n = w.shape[0]
        dense_bwd = torch.ops.aten.embedding_dense_backward
        sink = getattr(w, "main_grad", None)
        if sink is None:
            return None, dense_bwd(dy, tokens, n, -1, False)
        if w._mxk_grad_fresh:
            dense_bwd.out(dy, tokens, n, -1, False, out=sink)
            w._mxk_grad_fresh = False
        else:
            sink.add_(dense_bwd(dy, tokens, n, -1, False))
        _notify_grad(w)
        return None, None


class Embedding(nn.Embedding):
    """``nn.Embedding`` (no padding index, no max-norm) with the
    direct-to-flat-buffer weight gradient."""

    def __init__(self, num_embeddings: int, embedding_dim: int, **kw):
        super().__init__(num_embeddings, embedding_dim, **kw)
        if self.padding_idx is not None or self.max_norm is not None or self.sparse:
            raise ValueError("mxk8s Embedding: padding_idx / max_norm / sparse not supported")
        self.weight._mxk_direct_grad = True

    def forward(self, tokens: torch.Tensor) -> torch.Tensor:
        return _EmbeddingFn.apply(tokens, self.weight)
