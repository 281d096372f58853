#!/usr/bin/env python3
"""Attention backward at the Llama-3-8B step shape with the RoPE backward
fused into the dQ / dK stores (mxk_attn_bwd_rope) against variant 9 followed
by the stand-alone RoPE passes (the unfused chain), and variant 9 alone (no
RoPE: the fused kernels' own cost).  Interleaved blocks after a 2 s warm-up;
fused vs unfused d(qkv) bit for bit."""
import math
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxk8s.ops import _lib  # noqa: E402
from mxk8s.ops import attention as A  # noqa: E402
from mxk8s.ops.fused import _rope_launch, rope_tables  # noqa: E402


def main():
    B, S, hq, hkv, hd = 8, 2048, 32, 8, 128
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(B, S, (hq + 2 * hkv) * hd, device=dev, generator=g).bfloat16()
    q = qkv[..., :hq * hd].view(B, S, hq, hd)
    k = qkv[..., hq * hd:(hq + hkv) * hd].view(B, S, hkv, hd)
    v = qkv[..., (hq + hkv) * hd:].view(B, S, hkv, hd)
    o, lse = A.attn_fwd(q, k, v, causal=True)
    dout = torch.randn(B, S, hq, hd, device=dev, generator=g).bfloat16()
    cos, sin = rope_tables(S, hd, device=dev)
    L = _lib.lib()
    ws = torch.empty(L.mxk_attn_bwd_workspace_variant(B, S, hq, 9) // 4, dtype=torch.float32, device=dev)
    scale = 1.0 / math.sqrt(hd)

    def slices(buf):
        return (buf[..., :hq * hd].view(B, S, hq, hd), buf[..., hq * hd:(hq + hkv) * hd].view(B, S, hkv, hd),
                buf[..., (hq + hkv) * hd:].view(B, S, hkv, hd))

    fa, fb, fc = torch.empty_like(qkv), torch.empty_like(qkv), torch.empty_like(qkv)

    def fused():
        dq, dk, dv = slices(fa)
        st = L.mxk_attn_bwd_rope(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), dout.data_ptr(),
                                 lse.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), ws.data_ptr(),
                                 B, S, hq, hkv, hd, q.stride(1), k.stride(1), v.stride(1), dq.stride(1),
                                 dk.stride(1), dv.stride(1), cos.data_ptr(), sin.data_ptr(), scale, 1,
                                 _lib.stream_ptr(dev))
        assert st == 0, st

    def unfused():
        dq, dk, dv = slices(fb)
        gq, _, _ = A.attn_bwd(q, k, v, o, lse, dout, causal=True, dk=dk, dv=dv, variant=9)
        _rope_launch(gq, cos, sin, -1.0, out=dq)
        _rope_launch(dk, cos, sin, -1.0, out=dk)

    def plain():
        dq, dk, dv = slices(fc)
        A.attn_bwd(q, k, v, o, lse, dout, causal=True, dk=dk, dv=dv, variant=9)

    fused()
    unfused()
    print(f"RESULT fused bit-identical to unfused: {torch.equal(fa, fb)}", flush=True)
    runs = {"fused": fused, "unfused": unfused, "plain_v9": plain}
    if os.environ.get("ALT"):
        # the fused call from another build of the library (in-process A/B)
        import ctypes
        alt = ctypes.CDLL(os.environ["ALT"], mode=ctypes.RTLD_LOCAL)
        fn = alt.mxk_attn_bwd_rope
        fn.restype, fn.argtypes = _lib._SIGNATURES["mxk_attn_bwd_rope"]
        fd = torch.empty_like(qkv)

        def fused_alt():
            dq, dk, dv = slices(fd)
            st = fn(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), dout.data_ptr(),
                    lse.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), ws.data_ptr(), B, S, hq,
                    hkv, hd, q.stride(1), k.stride(1), v.stride(1), dq.stride(1), dk.stride(1),
                    dv.stride(1), cos.data_ptr(), sin.data_ptr(), scale, 1, _lib.stream_ptr(dev))
            assert st == 0, st

        fused_alt()
        print(f"RESULT fused bit-identical to fused_alt: {torch.equal(fa, fd)}", flush=True)
        runs["fused_alt"] = fused_alt
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 2.0:
        for f in runs.values():
            f()
        torch.cuda.synchronize()
    ts = {n: [] for n in runs}
    for _ in range(15):
        for n, f in runs.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(5):
                f()
            e.record()
            e.synchronize()
            ts[n].append(s.elapsed_time(e) / 5)
    for n, t in ts.items():
        print(f"RESULT {n} ms={statistics.median(t):.4f} min={min(t):.4f}", flush=True)


if __name__ == "__main__":
    main()
