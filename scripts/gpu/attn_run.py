#!/usr/bin/env python3
"""Attention forward + backward on the Llama-3-8B step shape, a few
iterations (for rocprofv3 counter passes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxk8s.ops import attention as A  # noqa: E402

B, S, Hq, Hkv, D = int(os.environ.get("B", 8)), 2048, 32, 8, 128
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
qkv = torch.randn(B, S, (Hq + 2 * Hkv) * D, device=dev, generator=g).bfloat16()
q, k, v = qkv.split([Hq * D, Hkv * D, Hkv * D], dim=-1)
q, k, v = q.view(B, S, Hq, D), k.view(B, S, Hkv, D), v.view(B, S, Hkv, D)
dout = torch.randn(B, S, Hq, D, device=dev, generator=g).bfloat16()
fwd_variants = [int(x) for x in os.environ.get("FWD_VARIANTS", "4").split(",") if x]
bwd_variants = [int(x) for x in os.environ.get("BWD_VARIANTS", "5").split(",") if x]
for _ in range(int(os.environ.get("ITERS", 6))):
    for fv in fwd_variants:
        o, lse = A.attn_fwd(q, k, v, causal=True, variant=fv)
    for bv in bwd_variants:
        A.attn_bwd(q, k, v, o, lse, dout, variant=bv)
torch.cuda.synchronize()
print("done", flush=True)
