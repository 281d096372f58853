#!/usr/bin/env python3
"""Time the hand-written flash attention (fwd, and fwd+bwd once available)
against torch SDPA on the Llama-3-8B shape: B=1, Hq=32, Hkv=8, S=2048,
D=128, causal, bf16, random data.  Prints one RESULT json line per kernel.

Timing follows bench.py: the chip is warmed for >= WARM_S (2 s) of
back-to-back launches before the first entry and >= 0.3 s per entry, then
each entry is the median over 7 blocks of back-to-back launches bracketed by
one event pair (per-launch events let the host fall behind the GPU and put
an event packet between every two kernels)."""
import json
import os
import statistics
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxk8s.ops import attention as A  # noqa: E402


WARM_S = float(os.environ.get("WARM_S", 2.0))
_warm = {"done": False}


def _spin(fn, seconds):
    t0 = time.perf_counter()
    while True:
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        if time.perf_counter() - t0 >= seconds:
            return


def bench(fn, blocks=7, reps=20):
    if not _warm["done"]:          # the first entry must not time a cold chip
        _spin(fn, WARM_S)
        _warm["done"] = True
    _spin(fn, 0.3)
    ts = []
    for _ in range(blocks):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) / reps)
    return statistics.median(ts)


def main():
    dev = torch.device("cuda")
    B, Hq, Hk, S, D = int(os.environ.get("BATCH", 1)), 32, 8, int(os.environ.get("SEQ", 2048)), 128
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(B, S, Hq, D, device=dev, generator=g).bfloat16()
    k = torch.randn(B, S, Hk, D, device=dev, generator=g).bfloat16()
    v = torch.randn(B, S, Hk, D, device=dev, generator=g).bfloat16()
    flops_fwd = 4 * B * Hq * S * S * D / 2
    res = {}
    res["mxk_fwd"] = bench(lambda: A.attn_fwd(q, k, v, causal=True))
    res["mxk_fwd_v0"] = bench(lambda: A.attn_fwd(q, k, v, causal=True, variant=0))
    res["mxk_fwd_v2"] = bench(lambda: A.attn_fwd(q, k, v, causal=True, variant=2))
    res["mxk_fwd_v4"] = bench(lambda: A.attn_fwd(q, k, v, causal=True, variant=4))
    res["mxk_fwd_v10"] = bench(lambda: A.attn_fwd(q, k, v, causal=True, variant=10))
    qt, kt, vt = (t.transpose(1, 2) for t in (q, k, v))
    with torch.no_grad():
        res["sdpa_fwd"] = bench(lambda: F.scaled_dot_product_attention(qt, kt, vt, is_causal=True,
                                                                      enable_gqa=True))
    o, lse = A.attn_fwd(q, k, v, causal=True)
    do = torch.randn_like(o)
    res["mxk_bwd"] = bench(lambda: A.attn_bwd(q, k, v, o, lse, do, causal=True))
    res["mxk_bwd_v3"] = bench(lambda: A.attn_bwd(q, k, v, o, lse, do, causal=True, variant=3))
    res["mxk_bwd_v5"] = bench(lambda: A.attn_bwd(q, k, v, o, lse, do, causal=True, variant=5))
    res["mxk_bwd_v6"] = bench(lambda: A.attn_bwd(q, k, v, o, lse, do, causal=True, variant=6))
    res["mxk_bwd_v7"] = bench(lambda: A.attn_bwd(q, k, v, o, lse, do, causal=True, variant=7))
    res["mxk_bwd_v8"] = bench(lambda: A.attn_bwd(q, k, v, o, lse, do, causal=True, variant=8))
    res["mxk_bwd_v9"] = bench(lambda: A.attn_bwd(q, k, v, o, lse, do, causal=True, variant=9))
    qg, kg, vg = (t.detach().transpose(1, 2).requires_grad_() for t in (q, k, v))
    dot = do.transpose(1, 2)

    def sdpa_fb():
        out = F.scaled_dot_product_attention(qg, kg, vg, is_causal=True, enable_gqa=True)
        out.backward(dot)
    res["sdpa_fwd_bwd"] = bench(sdpa_fb)
    def mxk_fb():
        o_, l_ = A.attn_fwd(q, k, v, causal=True)
        A.attn_bwd(q, k, v, o_, l_, do, causal=True)
    res["mxk_fwd_bwd"] = bench(mxk_fb)
    # useful FLOPs: fwd 2 products, bwd 5 products (causal halves all)
    def mult(name):
        return 3.5 if name.endswith("fwd_bwd") else 2.5 if "_bwd" in name else 1.0
    for name, ms in res.items():
        print("RESULT " + json.dumps({"kernel": name, "ms": round(ms, 4), "S": S, "B": B,
                                      "tflops": round(mult(name) * flops_fwd / ms / 1e9, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
