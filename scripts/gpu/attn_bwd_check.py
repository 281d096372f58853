#!/usr/bin/env python3
"""Cross-check of the two attention-backward variants on the Llama shape."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxk8s.ops import attention as A  # noqa: E402


def main():
    dev = torch.device("cuda")
    for (B, S, Hq, Hkv) in [(1, 2048, 32, 8), (2, 1024, 32, 8), (1, 512, 8, 2)]:
        D = 128
        g = torch.Generator(device=dev).manual_seed(0)
        qkv = torch.randn(B, S, (Hq + 2 * Hkv) * D, device=dev, generator=g).bfloat16()
        q, k, v = qkv.split([Hq * D, Hkv * D, Hkv * D], dim=-1)
        q, k, v = q.view(B, S, Hq, D), k.view(B, S, Hkv, D), v.view(B, S, Hkv, D)
        o, lse = A.attn_fwd(q, k, v, causal=True)
        dout = torch.randn(B, S, Hq, D, device=dev, generator=g).bfloat16()
        r0 = A.attn_bwd(q, k, v, o, lse, dout, variant=0)
        r1 = A.attn_bwd(q, k, v, o, lse, dout, variant=1)
        for name, a, b in zip(("dq", "dk", "dv"), r0, r1):
            d = (a.float() - b.float()).abs()
            print(f"B={B} S={S} Hq={Hq} Hkv={Hkv} {name}: max|v0-v1|={d.max().item():.4g} "
                  f"max|v0|={a.float().abs().max().item():.4g} nan={torch.isnan(b).any().item()}",
                  flush=True)


if __name__ == "__main__":
    main()
