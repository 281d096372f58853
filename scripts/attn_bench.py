#!/usr/bin/env python3
"""Time SDPA variants for the Llama-3-8B attention shape (fwd+bwd), bf16,
random data: B=1, Hq=32, Hkv=8, S=2048, D=128, causal."""
import statistics
import time

import torch
import torch.nn.functional as F


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
        s.record(); fn(); e.record(); e.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


def main():
    dev = torch.device("cuda")
    B, Hq, Hk, S, D = 1, 32, 8, 2048, 128
    q = torch.randn(B, Hq, S, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, Hk, S, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, Hk, S, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(B, Hq, S, D, device=dev, dtype=torch.bfloat16)
    flops_fwd = 4 * B * Hq * S * S * D / 2
    from torch.nn.attention import sdpa_kernel, SDPBackend

    def gqa():
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True)
        o.backward(do)

    def rep():
        kk = k.repeat_interleave(Hq // Hk, dim=1)
        vv = v.repeat_interleave(Hq // Hk, dim=1)
        o = F.scaled_dot_product_attention(q, kk, vv, is_causal=True)
        o.backward(do)

    def fwd_only():
        with torch.no_grad():
            F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True)

    res = {}
    for name, fn in [("gqa_default", gqa), ("repeat_kv_default", rep), ("fwd_only_gqa", fwd_only)]:
        try:
            res[name] = bench(fn)
        except Exception as e:
            res[name] = f"error {e}"[:100]
    for be in (SDPBackend.FLASH_ATTENTION, SDPBackend.EFFICIENT_ATTENTION, SDPBackend.CUDNN_ATTENTION):
        for name, fn in [("gqa", gqa), ("repeat_kv", rep)]:
            try:
                with sdpa_kernel([be]):
                    res[f"{name}_{be.name}"] = bench(fn)
            except Exception as e:
                res[f"{name}_{be.name}"] = f"error {str(e)[:80]}"
    for k_, v_ in res.items():
        if isinstance(v_, float):
            f = flops_fwd * (1 if "fwd_only" in k_ else 3.5)
            print(f"{k_:32s} {v_:8.3f} ms  {f / v_ / 1e9:8.1f} TF/s")
        else:
            print(f"{k_:32s} {v_}")


if __name__ == "__main__":
    main()
