"""Flat mixed-precision AdamW over a :class:`~mxk8s.parallel.ddp.FlatParamSpace`.

bf16 parameters + bf16 gradients (what RCCL moves), fp32 master weights and
moments.  On GPU the whole step is three HIP launches
(``native/kernels/optim.hip``): grad sum-of-squares, clip coefficient (folds
in the 1/world DDP average), fused AdamW over the decay region and over the
no-decay region — no host synchronisation.  On CPU the same math runs in
torch (the reference path the tests compare the kernel against).
"""
from __future__ import annotations

import torch

from ..ops import _lib
from .ddp import FlatParamSpace


class FlatAdamW:
    def __init__(self, space: FlatParamSpace, lr: float = 3e-4, betas=(0.9, 0.95),
                 eps: float = 1e-8, weight_decay: float = 0.1, max_grad_norm: float = 1.0,
                 grad_scale: float = 1.0):
        self.space = space
        self.lr, self.b1, self.b2, self.eps = lr, betas[0], betas[1], eps
        self.wd = weight_decay
        self.max_grad_norm = max_grad_norm
        self.grad_scale = grad_scale
        self.step_count = 0
        dev = space.param_buf.device
        self.master = space.param_buf.float().clone()
        self.exp_avg = torch.zeros_like(self.master)
        self.exp_avg_sq = torch.zeros_like(self.master)
        self._scale = torch.ones(2, dtype=torch.float32, device=dev)   # [scale, grad norm]
        if dev.type == "cuda":
            n_part = _lib.lib().mxk_sumsq_partials(space.numel)
            self._partials = torch.zeros(n_part, dtype=torch.float32, device=dev)

    @property
    def last_grad_norm(self) -> torch.Tensor:
        """Norm of the averaged gradient at the last step (device scalar)."""
        return self._scale[1]

    def _regions(self):
        n, nd = self.space.numel, self.space.n_decay
        return [(0, nd, self.wd), (nd, n, 0.0)]

    @torch.no_grad()
    def step(self) -> None:
        self.step_count += 1
        sp = self.space
        if sp.param_buf.device.type == "cuda":
            L = _lib.lib()
            s = _lib.stream_ptr(sp.param_buf.device)
            st = L.mxk_grad_clip_scale(sp.grad_buf.data_ptr(), sp.numel, self._partials.data_ptr(),
                                       float(self.grad_scale), float(self.max_grad_norm),
                                       self._scale.data_ptr(), s)
            _lib.check(st, "mxk_grad_clip_scale")
            esz, fsz = sp.param_buf.element_size(), 4
            for a, b, wd in self._regions():
                if b <= a:
                    continue
                st = L.mxk_adamw_bf16(sp.param_buf.data_ptr() + a * esz,
                                      self.master.data_ptr() + a * fsz,
                                      self.exp_avg.data_ptr() + a * fsz,
                                      self.exp_avg_sq.data_ptr() + a * fsz,
                                      sp.grad_buf.data_ptr() + a * esz, b - a, float(self.lr),
                                      float(self.b1), float(self.b2), float(self.eps), float(wd),
                                      self.step_count, self._scale.data_ptr(), s)
                _lib.check(st, "mxk_adamw_bf16")
            return
        self._step_reference()

    def _step_reference(self) -> None:
        sp = self.space
        g = sp.grad_buf.float()
        norm = g.norm() * self.grad_scale
        clip = 1.0
        if self.max_grad_norm > 0 and norm > self.max_grad_norm:
            clip = self.max_grad_norm / (norm + 1e-6)
        g = g * (self.grad_scale * clip)
        self._scale[0] = self.grad_scale * clip
        self._scale[1] = norm
        bc1 = 1 - self.b1 ** self.step_count
        bc2 = 1 - self.b2 ** self.step_count
        for a, b, wd in self._regions():
            if b <= a:
                continue
            p, m, v, gg = self.master[a:b], self.exp_avg[a:b], self.exp_avg_sq[a:b], g[a:b]
            p.mul_(1 - self.lr * wd)
            m.mul_(self.b1).add_(gg, alpha=1 - self.b1)
            v.mul_(self.b2).addcmul_(gg, gg, value=1 - self.b2)
            denom = v.sqrt() / (bc2 ** 0.5) + self.eps
            p.addcdiv_(m, denom, value=-self.lr / bc1)
        sp.param_buf.copy_(self.master.to(sp.param_buf.dtype))
