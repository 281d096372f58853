#!/usr/bin/env python3
"""In-process A/B of the attention backward (MODE=fwd: the forward,
FWD_VARIANT) between the default kernel
library and an alternative build (ALT=path.so, loaded beside it with
RTLD_LOCAL): interleaved timing blocks on the same clock, outputs compared
bit for bit.  Llama-3-8B step shape (B 8, S 2048, 32 q / 8 kv heads,
causal, fused QKV layout)."""
import ctypes
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxk8s.ops import _lib  # noqa: E402
from mxk8s.ops import attention as A  # noqa: E402


def main():
    B, S, Hq, Hkv, D = int(os.environ.get("B", 8)), 2048, 32, 8, 128
    variant = int(os.environ.get("VARIANT", 9))
    base = _lib.lib()
    alt = ctypes.CDLL(os.environ["ALT"], mode=ctypes.RTLD_LOCAL)
    for name, (res, args) in _lib._SIGNATURES.items():
        if hasattr(alt, name):
            fn = getattr(alt, name)
            fn.restype = res
            fn.argtypes = args
    libs = {"default": base, "alt": alt}
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(B, S, (Hq + 2 * Hkv) * D, device=dev, generator=g).bfloat16()
    q, k, v = qkv.split([Hq * D, Hkv * D, Hkv * D], dim=-1)
    q, k, v = q.view(B, S, Hq, D), k.view(B, S, Hkv, D), v.view(B, S, Hkv, D)
    o, lse = A.attn_fwd(q, k, v, causal=True)
    dout = torch.randn(B, S, Hq, D, device=dev, generator=g).bfloat16()

    fwd = os.environ.get("MODE", "bwd") == "fwd"

    def run(name):
        _lib._lib = libs[name]
        if fwd:
            return A.attn_fwd(q, k, v, causal=True, variant=int(os.environ.get("FWD_VARIANT", 4)))
        return A.attn_bwd(q, k, v, o, lse, dout, variant=variant)

    outs = {n: [x.clone() for x in run(n)] for n in libs}
    same = all(torch.equal(x, y) for x, y in zip(outs["default"], outs["alt"]))
    print(f"RESULT default bit-identical to alt: {same}", flush=True)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 2.0:
        for n in libs:
            run(n)
        torch.cuda.synchronize()
    ts = {n: [] for n in libs}
    for _ in range(int(os.environ.get("ROUNDS", 20))):
        for n in libs:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                run(n)
            e.record()
            e.synchronize()
            ts[n].append(s.elapsed_time(e) / 5)
    _lib._lib = base
    for n, t in ts.items():
        print(f"RESULT lib={n} variant={variant} ms={statistics.median(t):.4f} "
              f"min={min(t):.4f}", flush=True)
    r = [a / b for a, b in zip(ts["default"], ts["alt"])]
    print(f"RESULT default/alt per-round ratio median {statistics.median(r):.4f} "
          f"(min {min(r):.4f}, max {max(r):.4f})", flush=True)


if __name__ == "__main__":
    main()
