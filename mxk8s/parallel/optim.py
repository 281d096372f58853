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

        self._stages = None      # overlap: [(ranges, module)] in forward-need order
        self._events: list = []

    @property
    def last_grad_norm(self) -> torch.Tensor:
        """Norm of the averaged gradient at the last step (device scalar)."""
        return self._scale[1]

    # ------------------------------------------------------------------
    # Overlap with the next forward (GPU, unsharded).  AdamW is HBM-bound
    # (28 B/param, ~38 ms per Llama-3-8B step) and the forward is GEMM-bound,
    # so the update runs on a side stream in the order the forward needs the
    # parameters - stage 0 first, then one stage per module - and each module's
    # forward pre-hook makes the compute stream wait for its own stage only.
    # The clip coefficient needs every gradient, so the side stream starts
    # after the clip kernel; the compute stream waits for stage 0 before
    # step() returns (zero_grad then clears gradients stage 0 has read).
    def enable_overlap(self, stages) -> bool:
        """``stages``: list of (params, module-or-None) in forward order; the
        module's forward pre-hook waits for that stage's update.  Every
        parameter of the space must appear in exactly one stage."""
        sp = self.space
        if sp.param_buf.device.type != "cuda":
            return False
        index = {id(p): i for i, p in enumerate(sp.params)}
        seen = set()
        plan = []
        for params, module in stages:
            ranges = []
            for p in params:
                i = index[id(p)]
                if i in seen:
                    raise ValueError("parameter in two overlap stages")
                seen.add(i)
                a = sp.offsets[i]
                ranges.append((a, a + p.numel()))
            plan.append((self._merge_ranges(sorted(ranges)), module))
        if len(seen) != len(sp.params):
            raise ValueError(f"overlap stages cover {len(seen)} of {len(sp.params)} parameters")
        self._stages = plan
        self._side = torch.cuda.Stream(device=sp.param_buf.device)
        self._clip_done = torch.cuda.Event()
        self._events = [None] * len(plan)
        self._stage_events = [torch.cuda.Event() for _ in plan]
        for k, (_, module) in enumerate(plan):
            if module is not None:
                module.register_forward_pre_hook(lambda mod, args, k=k: self._wait_stage(k))
        return True

    def _merge_ranges(self, ranges):
        """Merge ranges separated only by alignment padding, never across the
        weight-decay boundary."""
        nd = self.space.n_decay
        out = []
        for a, b in ranges:
            if out and a - out[-1][1] < 64 and (out[-1][0] < nd) == (a < nd):
                out[-1] = (out[-1][0], b)
            else:
                out.append((a, b))
        return out

    def _wait_stage(self, k: int) -> None:
        ev = self._events[k]
        if ev is not None:
            torch.cuda.current_stream(self.space.param_buf.device).wait_event(ev)
            self._events[k] = None

    def synchronize(self) -> None:
        """Make the compute stream wait for every pending update (before
        reading parameters or optimizer state outside a forward)."""
        for k in range(len(self._events)):
            self._wait_stage(k)

    def _adamw_launch(self, L, a: int, b: int, stream: int) -> None:
        sp = self.space
        esz, fsz = sp.param_buf.element_size(), 4
        wd = self.wd if a < sp.n_decay else 0.0
        st = L.mxk_adamw_bf16(sp.param_buf.data_ptr() + a * esz,
                              self.master.data_ptr() + a * fsz,
                              self.exp_avg.data_ptr() + a * fsz,
                              self.exp_avg_sq.data_ptr() + a * fsz,
                              sp.grad_buf.data_ptr() + a * esz, b - a, float(self.lr),
                              float(self.b1), float(self.b2), float(self.eps), float(wd),
                              self.step_count, self._scale.data_ptr(), stream)
        _lib.check(st, "mxk_adamw_bf16")

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
            if self._stages is not None:
                self.synchronize()   # a stage never consumed by a forward
                dev = sp.param_buf.device
                main = torch.cuda.current_stream(dev)
                self._clip_done.record(main)
                self._side.wait_event(self._clip_done)
                side = self._side.cuda_stream
                for k, (ranges, _) in enumerate(self._stages):
                    for a, b in ranges:
                        self._adamw_launch(L, a, b, side)
                    self._stage_events[k].record(self._side)
                    self._events[k] = self._stage_events[k]
                self._wait_stage(0)
                return
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


class ShardedFlatAdamW:
    """ZeRO-1 AdamW for a :class:`~mxk8s.parallel.ddp.FlatDDP` built with
    ``shard_optimizer=True``.

    State per rank: fp32 master / exp_avg / exp_avg_sq for the rank's chunk
    of every bucket only (shard-local layout = the chunks in bucket order, the
    same layout as ``ddp.grad_shard``).  A step:

      1. sum of squares of the local gradient shard -> all-reduce of ONE fp32
         -> clip scale (device scalar, folds in 1/world; no host sync);
      2. per bucket: fused AdamW over the rank's chunk (split where the chunk
         crosses the no-weight-decay boundary), writing the bf16 parameters
         in place into the rank's chunk of ``param_buf``, then an async
         in-place all-gather of that bucket — the all-gather of bucket b runs
         on the RCCL stream while AdamW of bucket b+1 runs;
      3. the compute stream waits on every all-gather (no host sync) — or,
         with :meth:`enable_overlap`, each module's forward pre-hook waits for
         the all-gathers of just the buckets holding its parameters, and the
         buckets are updated + gathered in the order the forward needs them:
         the 16 GB (Llama-3-8B) parameter all-gather then runs under the
         next forward instead of in front of it.
    """

    def __init__(self, ddp, lr: float = 3e-4, betas=(0.9, 0.95), eps: float = 1e-8,
                 weight_decay: float = 0.1, max_grad_norm: float = 1.0):
        if not ddp.sharded:
            raise ValueError("ShardedFlatAdamW needs FlatDDP(shard_optimizer=True) with world > 1")
        import torch.distributed as dist
        self._dist = dist
        self.ddp = ddp
        sp = ddp.space
        self.lr, self.b1, self.b2, self.eps = lr, betas[0], betas[1], eps
        self.wd = weight_decay
        self.max_grad_norm = max_grad_norm
        self.step_count = 0
        dev = sp.param_buf.device
        # shard-local segments (shard_lo, flat_lo, n, wd): chunks split at n_decay
        self.segments = []
        for b in ddp.buckets:
            lo, hi = ddp.shard_range(b)
            cuts = [lo] + ([sp.n_decay] if lo < sp.n_decay < hi else []) + [hi]
            for a, z in zip(cuts[:-1], cuts[1:]):
                self.segments.append((b, b.shard_off + (a - lo), a, z - a,
                                      self.wd if a < sp.n_decay else 0.0))
        self.master = torch.empty(ddp.shard_numel, dtype=torch.float32, device=dev)
        for b in ddp.buckets:
            lo, hi = ddp.shard_range(b)
            self.master[b.shard_off:b.shard_off + hi - lo].copy_(sp.param_buf[lo:hi].float())
        self.exp_avg = torch.zeros_like(self.master)
        self.exp_avg_sq = torch.zeros_like(self.master)
        self._scale = torch.ones(2, dtype=torch.float32, device=dev)   # [scale, grad norm]
        self._sumsq = torch.zeros(1, dtype=torch.float32, device=dev)
        if dev.type == "cuda":
            n_part = _lib.lib().mxk_sumsq_partials(ddp.shard_numel)
            self._partials = torch.zeros(n_part, dtype=torch.float32, device=dev)
        self._order = list(range(len(ddp.buckets)))     # bucket update / gather order
        self._pending: dict[int, object] = {}           # bucket index -> all-gather handle
        self._module_buckets: list = []                 # per hooked module: bucket indices
        self.waits: list[int] = []                      # bucket indices as waited (tests)

    @property
    def last_grad_norm(self) -> torch.Tensor:
        return self._scale[1]

    def enable_overlap(self, stages) -> bool:
        """``stages``: [(params, module)] in the order the forward needs the
        parameters (``mxk8s.train.ddp_llama.overlap_stages``: the embedding
        with every 1-D weight first — the fused norms read the next layer's
        weight a layer early — then each block, then the LM head); every
        trainable parameter in exactly one stage.  Buckets are then updated
        and all-gathered in first-need order, and the module's forward
        pre-hook waits for the buckets holding its stage's parameters only."""
        ddp = self.ddp
        bucket_of = {}
        for i, b in enumerate(ddp.buckets):
            for p in b.params:
                bucket_of[id(p)] = i
        need, first, seen = [], {}, 0
        for k, (params, _) in enumerate(stages):
            idx = sorted({bucket_of[id(p)] for p in params})
            seen += len(params)
            need.append(idx)
            for i in idx:
                first.setdefault(i, k)
        if seen != len(ddp.space.params) or len(first) != len(ddp.buckets):
            raise ValueError(f"overlap stages cover {seen} of {len(ddp.space.params)} parameters")
        self._order = sorted(range(len(ddp.buckets)), key=lambda i: (first[i], i))
        self._module_buckets = need
        for k, (_, module) in enumerate(stages):
            module.register_forward_pre_hook(
                lambda mod, args, k=k: self._wait_buckets(self._module_buckets[k]))
        return True

    def _wait_buckets(self, idx) -> None:
        for i in idx:
            h = self._pending.pop(i, None)
            if h is not None:
                h.wait()
                self.waits.append(i)

    def synchronize(self) -> None:
        """Wait for every pending parameter all-gather (before reading the
        parameters outside a hooked forward: checkpoints, evaluation)."""
        self._wait_buckets(list(self._pending))

    def _clip(self) -> None:
        ddp = self.ddp
        g = ddp.grad_shard
        if g.device.type == "cuda":
            L = _lib.lib()
            s = _lib.stream_ptr(g.device)
            _lib.check(L.mxk_grad_sumsq(g.data_ptr(), g.numel(), self._partials.data_ptr(),
                                        self._sumsq.data_ptr(), s), "mxk_grad_sumsq")
            self._dist.all_reduce(self._sumsq, op=self._dist.ReduceOp.SUM, group=ddp.group)
            _lib.check(L.mxk_clip_scale_from_sumsq(self._sumsq.data_ptr(), 1.0 / ddp.world,
                                                   float(self.max_grad_norm),
                                                   self._scale.data_ptr(), s),
                       "mxk_clip_scale_from_sumsq")
            return
        self._sumsq[0] = g.float().pow(2).sum()
        self._dist.all_reduce(self._sumsq, op=self._dist.ReduceOp.SUM, group=ddp.group)
        norm = self._sumsq[0].sqrt() / ddp.world
        clip = 1.0
        if self.max_grad_norm > 0 and norm > self.max_grad_norm:
            clip = self.max_grad_norm / (norm + 1e-6)
        self._scale[0] = clip / ddp.world
        self._scale[1] = norm

    def _adamw_segment(self, so: int, flat_lo: int, n: int, wd: float) -> None:
        sp, ddp = self.ddp.space, self.ddp
        if sp.param_buf.device.type == "cuda":
            L = _lib.lib()
            esz, fsz = sp.param_buf.element_size(), 4
            st = L.mxk_adamw_bf16(sp.param_buf.data_ptr() + flat_lo * esz,
                                  self.master.data_ptr() + so * fsz,
                                  self.exp_avg.data_ptr() + so * fsz,
                                  self.exp_avg_sq.data_ptr() + so * fsz,
                                  ddp.grad_shard.data_ptr() + so * esz, n, float(self.lr),
                                  float(self.b1), float(self.b2), float(self.eps), float(wd),
                                  self.step_count, self._scale.data_ptr(),
                                  _lib.stream_ptr(sp.param_buf.device))
            _lib.check(st, "mxk_adamw_bf16")
            return
        bc1 = 1 - self.b1 ** self.step_count
        bc2 = 1 - self.b2 ** self.step_count
        g = ddp.grad_shard[so:so + n].float() * self._scale[0]
        p, m, v = self.master[so:so + n], self.exp_avg[so:so + n], self.exp_avg_sq[so:so + n]
        p.mul_(1 - self.lr * wd)
        m.mul_(self.b1).add_(g, alpha=1 - self.b1)
        v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
        p.addcdiv_(m, v.sqrt() / (bc2 ** 0.5) + self.eps, value=-self.lr / bc1)
        sp.param_buf[flat_lo:flat_lo + n].copy_(p.to(sp.param_buf.dtype))

    @torch.no_grad()
    def step(self) -> None:
        self.synchronize()      # a bucket no forward consumed (its chunk is rewritten below)
        self.step_count += 1
        ddp, sp = self.ddp, self.ddp.space
        self._clip()
        segs: dict[int, list] = {}
        index = {id(b): i for i, b in enumerate(ddp.buckets)}
        for seg in self.segments:
            segs.setdefault(index[id(seg[0])], []).append(seg)
        for i in self._order:
            b = ddp.buckets[i]
            for _, so, lo, n, wd in segs.get(i, []):
                self._adamw_segment(so, lo, n, wd)
            lo, hi = ddp.shard_range(b)
            self._pending[i] = self._dist.all_gather_into_tensor(
                sp.param_buf[b.start:b.end], sp.param_buf[lo:hi], group=ddp.group, async_op=True)
        if not self._module_buckets:
            self.synchronize()  # no overlap: every parameter is whole when step() returns
