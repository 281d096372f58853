#!/usr/bin/env python3
"""Cycle anatomy of the variant-9 dQ kernel (attention_dq256.hip): the
diagnostic instance (mxk_attn_bwd_dq256_stamps) adds up each wave's shader
cycles in its prologue, phases A (S^T / dP^T beside the g1 softmax), phases B
(dQ^T beside the g0 softmax), the per-tile barrier + DMA issue, and the tail.
Llama-3-8B step shape (B 8, S 2048, Hq 32, Hkv 8, causal).  Prints the sums
per 32-key step (the MFMA floor of a step is 48 x 32 = 1536 cycles)."""
import math
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
o, lse = A.attn_fwd(q, k, v, causal=True)
scale = 1 / math.sqrt(D)
dq = torch.empty_like(q)
rowc = torch.empty(B, Hq, S, 2, device=dev)
nwg = B * (Hq // 4) * (S // 64)
st = torch.zeros(nwg * 4 * 9, dtype=torch.int64, device=dev)
L = _lib.lib()
for _ in range(3):
    rc = L.mxk_attn_bwd_dq256_stamps(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(),
                                     do.data_ptr(), lse.data_ptr(), dq.data_ptr(), rowc.data_ptr(),
                                     B, S, Hq, Hkv, q.stride(1), k.stride(1), v.stride(1), scale,
                                     st.data_ptr(), _lib.stream_ptr(dev))
    assert rc == 0, rc
torch.cuda.synchronize()
x = st.view(nwg, 4, 9).double().cpu()
x = x[x[:, 0, 0] > 0]          # the persistent launch fills one row per CU
# steps per workgroup: the work order is XCD-remapped, so derive it from the
# stamps' own phase-A count is not possible; sum over the grid instead
steps = B * (Hq // 4) * sum(2 * (qb + 1) for qb in range(S // 64))
tot = x.sum(dim=(0, 1))
names = ["total", "prologue rest", "phase A", "phase B", "barrier", "tail+store",
         "load issue", "wait dO/O", "delta+wait Q"]
print(f"workgroups {nwg}, 32-key steps {steps} (x4 waves)")
for i, n in enumerate(names[:9]):
    print(f"  {n:12s} {tot[i].item() / (4 * steps):9.1f} cycles per step per wave   "
          f"({100 * tot[i].item() / tot[0].item():5.1f} %)")
wt = x[:, :, 0]
print(f"  wave time: max {wt.max().item():.0f}  median {wt.median().item():.0f}  "
      f"min {wt.min().item():.0f} cycles")
