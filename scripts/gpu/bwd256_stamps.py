#!/usr/bin/env python3
"""Cycle anatomy of the 256-key dK / dV kernel (backward variant 6's second
kernel): the diagnostic instance (mxk_attn_bwd_dkdv256_stamps) adds up each
wave's shader cycles in the step phases A (S / dP of key tile 0), B (S / dP
of tile 1 beside softmax 0), C (dK / dV of tile 0 beside softmax 1), D (dK /
dV of tile 1) and the end-of-step wait + barrier.  Llama-3-8B step shape
(B 8, S 2048, Hq 32, Hkv 8, causal).  rowc is synthetic (-lse / scale from
the forward, delta = 0): timing only."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxk8s.ops import _lib  # noqa: E402
from mxk8s.ops import attention as A  # noqa: E402

B, S, Hq, Hkv, D = int(os.environ.get("B", 8)), 2048, 32, 8, 128
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
q = torch.randn(B, S, Hq, D, device=dev, generator=g).bfloat16()
k = torch.randn(B, S, Hkv, D, device=dev, generator=g).bfloat16()
v = torch.randn(B, S, Hkv, D, device=dev, generator=g).bfloat16()
do = torch.randn(B, S, Hq, D, device=dev, generator=g).bfloat16()
scale = D ** -0.5
_, lse = A.attn_fwd(q, k, v, causal=True)
rowc = torch.stack([-lse / scale, torch.zeros_like(lse)], dim=-1).contiguous()
dk = torch.empty_like(k)
dv = torch.empty_like(v)
nwg = B * Hkv * (S // 256)
st = torch.zeros(nwg * 4 * 9, dtype=torch.int64, device=dev)
f = _lib.lib().mxk_attn_bwd_dkdv256_stamps
vp, i_, l_ = ctypes.c_void_p, ctypes.c_int, ctypes.c_long
f.restype = i_
f.argtypes = [vp, vp, vp, vp, vp, vp, vp, i_, i_, i_, i_, l_, l_, l_, l_, l_, ctypes.c_float, i_,
              vp, vp]
for _ in range(3):
    rc = f(q.data_ptr(), k.data_ptr(), v.data_ptr(), do.data_ptr(), rowc.data_ptr(), dk.data_ptr(),
           dv.data_ptr(), B, S, Hq, Hkv, Hq * D, Hkv * D, Hkv * D, Hkv * D, Hkv * D, scale, 1,
           st.data_ptr(), _lib.stream_ptr(dev))
    assert rc == 0, rc
torch.cuda.synchronize()
s = st.view(nwg, 4, 9).double().cpu()
tot = s[:, :, 0]
names = ["AB", "C(pending dkdv + softmax0)", "D(dkdv tile 0)", "copies", "wait+barrier",
         "prologue", "tail", "stores"]
share = {n: (s[:, :, 1 + e].sum() / tot.sum()).item() for e, n in enumerate(names)}
other = 1 - sum(share.values())
# steps: a key block kb of the (b, hkv) pair sweeps 4 heads x (S - 256 kb) / 32 slices
kb = torch.arange(nwg) // (B * Hkv)
steps = (4 * (S - 256 * kb) // 32).double()
per_step = {n: (s[:, :, 1 + e].sum(1) / 4 / steps).median().item() for e, n in enumerate(names[:5])}
print("share of wave cycles: " + ", ".join(f"{n} {v:.3f}" for n, v in share.items()) +
      f", other {other:.3f}")
print("median cycles per step (64 MFMAs = 2048 at the roof; AB 32 = 1024, C / D 16 = 512): " +
      ", ".join(f"{n} {v:.0f}" for n, v in per_step.items()))
print("median per wave: total %.0f, prologue %.0f, tail %.0f, stores %.0f cycles" % (
    tot.median().item(), s[:, :, 6].median().item(), s[:, :, 7].median().item(), s[:, :, 8].median().item()))
print("done", flush=True)
