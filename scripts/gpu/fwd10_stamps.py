#!/usr/bin/env python3
"""Forward variant 10 cycle anatomy: the diagnostic instance
(mxk_attn_fwd256_stamps) adds up each wave's shader cycles in phase 1
(S = K Q^T beside the softmax finish), phase 2 (O += V^T P^T beside the
softmax start) and the per-tile barrier (DMA wait + s_barrier).  Prints
medians per wave and per tile at the Llama-3-8B step shape (B 8, S 2048,
Hq 32, Hkv 8, causal)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxk8s.ops import _lib  # noqa: E402

B, S, Hq, Hkv, D = int(os.environ.get("B", 8)), 2048, 32, 8, 128
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
q = torch.randn(B, S, Hq, D, device=dev, generator=g).bfloat16()
k = torch.randn(B, S, Hkv, D, device=dev, generator=g).bfloat16()
v = torch.randn(B, S, Hkv, D, device=dev, generator=g).bfloat16()
o = torch.empty_like(q)
lse = torch.empty(B, Hq, S, device=dev)
nwg = B * Hq * (S // 256)
st = torch.zeros(nwg * 4 * 6, dtype=torch.int64, device=dev)
L = _lib.lib()
f = L.mxk_attn_fwd256_stamps
vp, i_, l_ = ctypes.c_void_p, ctypes.c_int, ctypes.c_long
f.restype = i_
f.argtypes = [vp, vp, vp, vp, vp, i_, i_, i_, i_, l_, l_, l_, ctypes.c_float, i_, vp, vp]
for causal in (1, 0):
    for _ in range(3):
        rc = f(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(), B, S, Hq, Hkv,
               Hq * D, Hkv * D, Hkv * D, D ** -0.5, causal, st.data_ptr(), _lib.stream_ptr(dev))
        assert rc == 0, rc
    torch.cuda.synchronize()
    s = st.view(nwg, 4, 6).float().cpu()
    qb = torch.arange(nwg) % (S // 256)        # block -> q block (not exact under the XCD map)
    tiles = 4 * (S // 256) if not causal else None
    tot, p1, p2, bar, pro, tail = (s[:, :, i] for i in range(6))
    print(f"causal={causal} median per wave: total {tot.median():.0f} cyc, phase1 {p1.median():.0f}, "
          f"phase2 {p2.median():.0f}, barrier {bar.median():.0f}, prologue {pro.median():.0f}, "
          f"tail {(tail - p1 - p2 - bar - pro).median():.0f}, epilogue {(tot - tail).median():.0f}")
    # per tile: the total tile count of a wave is J (causal: 4 (qb + 1))
    J = (p1 + p2 + bar).sum(1)
    print(f"   sum over waves: phase1 {p1.sum() / tot.sum():.3f}, phase2 {p2.sum() / tot.sum():.3f}, "
          f"barrier {bar.sum() / tot.sum():.3f} of total; max/median total {tot.max() / tot.median():.2f}")
    if not causal:
        nt = S // 64
        print(f"   per tile: phase1 {p1.median() / nt:.0f} cyc, phase2 {p2.median() / nt:.0f}, "
              f"barrier {bar.median() / nt:.0f} (64 MFMAs = 2048 cyc at the MFMA roof)")
print("done", flush=True)
