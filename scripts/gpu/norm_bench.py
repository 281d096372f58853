#!/usr/bin/env python3
"""RMSNorm backward (with and without the fused residual gradient) on the
Llama-3-8B step shape (16k tokens x 4096): ms and effective HBM GB/s."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxk8s.ops import _lib  # noqa: E402

T, H = int(os.environ.get("TOKENS", 16384)), 4096
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
r = lambda *s: torch.randn(*s, device=dev, generator=g).bfloat16()  # noqa: E731
dy, x, dres, w = r(T, H), r(T, H), r(T, H), r(H)
rstd = torch.rand(T, device=dev, generator=g) + 0.5
dx, dw = torch.empty_like(x), torch.empty_like(w)
L = _lib.lib()
ws = torch.empty(L.mxk_rmsnorm_bwd_workspace(T, H) // 4, dtype=torch.float32, device=dev)
for use_res in (False, True):
    def run():
        _lib.check(L.mxk_rmsnorm_bwd(dy.data_ptr(), x.data_ptr(), w.data_ptr(), rstd.data_ptr(),
                                     dres.data_ptr() if use_res else None, dx.data_ptr(),
                                     dw.data_ptr(), None, ws.data_ptr(), T, H,
                                     _lib.stream_ptr(dev)), "rmsnorm_bwd")
    for _ in range(5):
        run()
    ts = []
    for _ in range(30):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        run()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    t = statistics.median(ts)
    nbytes = T * H * 2 * (4 if use_res else 3)
    print(f"RESULT rmsnorm_bwd dres={use_res} ms={t:.4f} GB/s={nbytes / t / 1e6:.0f}", flush=True)
