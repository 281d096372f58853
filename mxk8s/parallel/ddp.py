"""Flat-buffer data parallelism over RCCL/xGMI with bucketed, backward-overlapped
all-reduce (BASELINE config 5; SURVEY.md §2.4 "N10 DDP gradient sync").

Design (MI355X-first rather than a copy of torch DDP's call pattern):

* every parameter is a view into ONE contiguous bf16 buffer and every
  gradient a view into ONE contiguous bf16 buffer, laid out in reverse
  registration order (= the order backward produces gradients); 1-D
  parameters (norm weights, no weight decay) go last;
* autograd accumulates straight into those views (``.grad`` is pre-set), so
  a bucket is a contiguous slice — no gather/scatter copies;
* a post-accumulate-grad hook counts arrivals per bucket and launches an async
  ``all_reduce`` (SUM, bf16 on the wire) the moment a bucket is complete, so
  RCCL rings run over xGMI while backward keeps computing;
* buckets default to 512 MiB: xGMI is point-to-point (7 links x ~153 GB/s per
  MI355X), ring collectives are per-link bound and want few, large messages;
  16 GB of Llama-3-8B bf16 gradients = ~32 buckets;
* the 1/world average and gradient clipping are folded into the fused
  optimizer kernel (``mxk8s.parallel.optim``), not applied as separate passes.

Works with any backend: ``nccl`` (= RCCL) on GPUs, ``gloo`` on CPU (tests).
"""
from __future__ import annotations

import contextlib
from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from . import dist as mxdist

ALIGN = 64   # elements: keeps every slot 16-B (bf16) and 32-B (fp32) aligned


class FlatParamSpace:
    """Contiguous bf16 (or any dtype) storage for all parameters and grads."""

    def __init__(self, module: nn.Module, dtype: Optional[torch.dtype] = None):
        params = [p for p in module.parameters() if p.requires_grad]
        if not params:
            raise ValueError("module has no trainable parameters")
        dev = params[0].device
        self.dtype = dtype or params[0].dtype
        # backward order ~ reverse registration order; 1-D (no-decay) last
        order = [p for p in reversed(params) if p.dim() >= 2] + \
                [p for p in reversed(params) if p.dim() < 2]
        self.params = order
        self.offsets = []
        off = 0
        n_decay = 0
        for p in order:
            self.offsets.append(off)
            off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
            if p.dim() >= 2:
                n_decay = off
        self.numel = off
        self.n_decay = n_decay
        self.param_buf = torch.zeros(self.numel, dtype=self.dtype, device=dev)
        self.grad_buf = torch.zeros(self.numel, dtype=self.dtype, device=dev)
        with torch.no_grad():
            for p, o in zip(order, self.offsets):
                view = self.param_buf[o:o + p.numel()].view_as(p)
                view.copy_(p.detach().to(self.dtype))
                p.data = view
                p.grad = self.grad_buf[o:o + p.numel()].view_as(p)

    def zero_grad(self) -> None:
        self.grad_buf.zero_()
        for p, o in zip(self.params, self.offsets):   # re-attach if someone set None
            if p.grad is None or p.grad.data_ptr() != self.grad_buf[o:].data_ptr():
                p.grad = self.grad_buf[o:o + p.numel()].view_as(p)


class Bucket:
    __slots__ = ("start", "end", "params", "pending", "handle", "launched")

    def __init__(self, start: int):
        self.start = start
        self.end = start
        self.params: list = []
        self.pending = 0
        self.handle = None
        self.launched = False


class FlatDDP:
    """Wraps a module whose parameters were flattened by :class:`FlatParamSpace`."""

    def __init__(self, module: nn.Module, bucket_mb: float = 512.0,
                 process_group=None, broadcast_from: Optional[int] = 0):
        self.module = module
        self.space = FlatParamSpace(module)
        self.group = process_group
        self.world = dist.get_world_size(process_group) if mxdist.active() else 1
        esz = self.space.param_buf.element_size()
        cap = max(1, int(bucket_mb * 2 ** 20 / esz))
        self.buckets: list[Bucket] = []
        cur = Bucket(0)
        self._bucket_of = {}
        for p, o in zip(self.space.params, self.space.offsets):
            n = (p.numel() + ALIGN - 1) // ALIGN * ALIGN
            if cur.params and (o + n - cur.start) > cap:
                self.buckets.append(cur)
                cur = Bucket(o)
            cur.params.append(p)
            cur.end = o + n
            self._bucket_of[id(p)] = cur
        self.buckets.append(cur)
        self._sync_enabled = True
        self._hooks = []
        if self.world > 1:
            if broadcast_from is not None:
                dist.broadcast(self.space.param_buf, src=broadcast_from, group=process_group)
            for p in self.space.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
        self._reset_buckets()

    # ------------------------------------------------------------------
    def _reset_buckets(self) -> None:
        for b in self.buckets:
            b.pending = len(b.params)
            b.handle = None
            b.launched = False

    def _launch(self, b: Bucket) -> None:
        if b.launched:
            return
        b.launched = True
        b.handle = dist.all_reduce(self.space.grad_buf[b.start:b.end], op=dist.ReduceOp.SUM,
                                   group=self.group, async_op=True)

    def _on_grad(self, p) -> None:
        if not self._sync_enabled:
            return
        b = self._bucket_of[id(p)]
        b.pending -= 1
        if b.pending == 0:
            self._launch(b)

    @contextlib.contextmanager
    def no_sync(self):
        """Gradient accumulation steps: accumulate locally, reduce later."""
        self._sync_enabled = False
        try:
            yield
        finally:
            self._sync_enabled = True

    def finish_grad_sync(self) -> None:
        """Launch any bucket that did not complete (unused params) and wait."""
        if self.world > 1:
            for b in self.buckets:
                if not b.launched:
                    self._launch(b)
            for b in self.buckets:
                if b.handle is not None:
                    b.handle.wait()
        self._reset_buckets()

    def zero_grad(self) -> None:
        self.space.zero_grad()

    def __call__(self, *a, **kw):
        return self.module(*a, **kw)

    @property
    def grad_scale(self) -> float:
        """Factor turning the SUM all-reduce into the mean gradient."""
        return 1.0 / self.world
