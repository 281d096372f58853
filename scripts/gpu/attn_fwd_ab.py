#!/usr/bin/env python3
"""A/B of the attention forward variants on the Llama-3-8B step shape
(B 8, S 2048, 32 q / 8 kv heads, fused QKV layout), interleaved rounds;
checks that the variants agree bit for bit."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxk8s.ops import attention as A  # noqa: E402


def main():
    B, S, Hq, Hkv, D = int(os.environ.get("B", 8)), int(os.environ.get("S", 2048)), 32, 8, 128
    variants = [int(x) for x in os.environ.get("VARIANTS", "0,2").split(",")]
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(B, S, (Hq + 2 * Hkv) * D, device=dev, generator=g).bfloat16()
    q, k, v = qkv.split([Hq * D, Hkv * D, Hkv * D], dim=-1)
    q, k, v = q.view(B, S, Hq, D), k.view(B, S, Hkv, D), v.view(B, S, Hkv, D)
    causal = os.environ.get("CAUSAL", "1") == "1"
    outs = {vv: A.attn_fwd(q, k, v, causal=causal, variant=vv) for vv in variants}
    for vv in variants[1:]:
        same = all(torch.equal(x, y) for x, y in zip(outs[variants[0]], outs[vv]))
        print(f"RESULT variant={vv} bit-identical to variant={variants[0]}: {same}", flush=True)
    fl = 4 * B * Hq * S * S * D / (2 if causal else 1)
    ts = {vv: [] for vv in variants}
    # time-floored warm-up (the clock ramps over ~1 s; bench.py's protocol)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < float(os.environ.get("WARM_S", 2.0)):
        for vv in variants:
            A.attn_fwd(q, k, v, causal=causal, variant=vv)
        torch.cuda.synchronize()
    for _ in range(10):
        for vv in variants:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                A.attn_fwd(q, k, v, causal=causal, variant=vv)
            e.record()
            e.synchronize()
            ts[vv].append(s.elapsed_time(e) / 5)
    for vv, t in ts.items():
        m = statistics.median(t[2:])
        print(f"RESULT fwd causal={int(causal)} variant={vv} B={B} ms={m:.4f} tflops={fl / m / 1e9:.1f}", flush=True)


if __name__ == "__main__":
    main()
