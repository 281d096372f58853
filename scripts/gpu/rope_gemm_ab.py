#!/usr/bin/env python3
"""The Llama-3-8B QKV projection (16384 x 6144 x 4096) with the rotary
embedding in its epilogue (mxk_gemm_bf16_rope) against the GEMM followed by
the stand-alone RoPE pass over q and k: interleaved timing blocks after a
2 s warm-up, outputs bit for bit."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxk8s.ops import _lib  # noqa: E402
from mxk8s.ops.fused import _rope_launch, rope_tables  # noqa: E402
from mxk8s.ops.gemm import gemm_bf16_tn  # noqa: E402


def main():
    B, S, dim, hq, hkv, hd = 8, 2048, 4096, 32, 8, 128
    N = (hq + 2 * hkv) * hd
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B * S, dim, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, dim, device=dev, generator=g) / 64).bfloat16()
    cos, sin = rope_tables(S, hd, device=dev)
    L = _lib.lib()

    def fused(out):
        st = L.mxk_gemm_bf16_rope(x.data_ptr(), w.data_ptr(), out.data_ptr(), B * S, N, dim, dim, dim,
                                  N, cos.data_ptr(), sin.data_ptr(), S, (hq + hkv) * hd,
                                  _lib.stream_ptr(dev))
        assert st == 0, st

    def unfused(out):
        gemm_bf16_tn(x, w, out)
        o3 = out.view(B, S, N)
        q = o3[..., :hq * hd].view(B, S, hq, hd)
        k = o3[..., hq * hd:(hq + hkv) * hd].view(B, S, hkv, hd)
        _rope_launch(q, cos, sin, 1.0, out=q)
        _rope_launch(k, cos, sin, 1.0, out=k)

    a = torch.empty(B * S, N, device=dev, dtype=torch.bfloat16)
    b = torch.empty_like(a)
    fused(a)
    unfused(b)
    print(f"RESULT fused bit-identical to GEMM + RoPE pass: {torch.equal(a, b)}", flush=True)
    runs = {"fused": lambda: fused(a), "unfused": lambda: unfused(b)}
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 2.0:
        for f in runs.values():
            f()
        torch.cuda.synchronize()
    ts = {n: [] for n in runs}
    for _ in range(20):
        for n, f in runs.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                f()
            e.record()
            e.synchronize()
            ts[n].append(s.elapsed_time(e) / 10)
    for n, t in ts.items():
        print(f"RESULT {n} ms={statistics.median(t):.4f} min={min(t):.4f}", flush=True)


if __name__ == "__main__":
    main()
