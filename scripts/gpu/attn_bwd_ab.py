#!/usr/bin/env python3
"""A/B of the attention backward variants on the Llama-3-8B step shape
(B 8, S 2048, 32 q / 8 kv heads, fused QKV layout), interleaved rounds."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxk8s.ops import attention as A  # noqa: E402


def main():
    B, S, Hq, Hkv, D = int(os.environ.get("B", 8)), 2048, 32, 8, 128
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(B, S, (Hq + 2 * Hkv) * D, device=dev, generator=g).bfloat16()
    q, k, v = qkv.split([Hq * D, Hkv * D, Hkv * D], dim=-1)
    q, k, v = q.view(B, S, Hq, D), k.view(B, S, Hkv, D), v.view(B, S, Hkv, D)
    o, lse = A.attn_fwd(q, k, v, causal=True)
    dout = torch.randn(B, S, Hq, D, device=dev, generator=g).bfloat16()
    fl = 2.5 * 4 * B * Hq * S * S * D / 2    # causal fwd FLOPs x 2.5
    variants = [int(x) for x in os.environ.get("VARIANTS", "0,1").split(",")]
    ts = {vv: [] for vv in variants}
    outs = {vv: A.attn_bwd(q, k, v, o, lse, dout, variant=vv) for vv in variants}
    for vv in variants[1:]:
        same = all(torch.equal(x, y) for x, y in zip(outs[variants[0]], outs[vv]))
        print(f"RESULT variant={vv} bit-identical to variant={variants[0]}: {same}", flush=True)
    # SAVE: the first variant's (dq, dk, dv) to a file; against a saved file
    # from another kernel library (MXK_KERNELS_LIB), bit for bit
    if os.environ.get("SAVE"):
        path = os.environ["SAVE"]
        cur = [x.cpu() for x in outs[variants[0]]]
        if os.path.exists(path):
            ref = torch.load(path, weights_only=True)
            same = all(torch.equal(x, y) for x, y in zip(cur, ref))
            print(f"RESULT variant={variants[0]} bit-identical to {path}: {same}", flush=True)
        else:
            torch.save(cur, path)
    # time-floored warm-up (the clock ramps over ~1 s; bench.py's protocol)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < float(os.environ.get("WARM_S", 2.0)):
        for vv in variants:
            A.attn_bwd(q, k, v, o, lse, dout, variant=vv)
        torch.cuda.synchronize()
    for _ in range(10):
        for vv in variants:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                A.attn_bwd(q, k, v, o, lse, dout, variant=vv)
            e.record()
            e.synchronize()
            ts[vv].append(s.elapsed_time(e) / 5)
    for vv, t in ts.items():
        m = statistics.median(t)
        print(f"RESULT variant={vv} B={B} ms={m:.4f} tflops={fl / m / 1e9:.1f}", flush=True)


if __name__ == "__main__":
    main()
