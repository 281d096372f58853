#!/usr/bin/env python3
"""Share of each k-iteration segment of the default GEMM schedule (diagnostic
build = variant 12 with s_memtime stamps; STAMP_VARIANT=14 stamps schedule 13): k-step 0, wait + barrier, k-step 1."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxk8s.ops import _lib  # noqa: E402


def main():
    n = int(os.environ.get("SIZE", 8192))
    variant = int(os.environ.get("STAMP_VARIANT", 12))
    dev = torch.device("cuda")
    L = _lib.lib()
    L.mxk_gemm_bf16_stamps.restype = ctypes.c_int
    L.mxk_gemm_bf16_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    g = torch.Generator(device=dev).manual_seed(0)
    A = (torch.rand(n, n, device=dev, generator=g) * 2 - 1).bfloat16()
    B = (torch.rand(n, n, device=dev, generator=g) * 2 - 1).bfloat16()
    C = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
    out = (ctypes.c_ulonglong * 4)()
    for _ in range(20):
        L.mxk_gemm_bf16_tn_variant(A.data_ptr(), B.data_ptr(), C.data_ptr(), n, n, n, n, n, n, variant,
                                   _lib.stream_ptr(dev))
    torch.cuda.synchronize()
    _lib.check(L.mxk_gemm_bf16_stamps(out, 1), "stamps reset")
    iters = 50
    for _ in range(iters):
        L.mxk_gemm_bf16_tn_variant(A.data_ptr(), B.data_ptr(), C.data_ptr(), n, n, n, n, n, n, variant,
                                   _lib.stream_ptr(dev))
    torch.cuda.synchronize()
    _lib.check(L.mxk_gemm_bf16_stamps(out, 0), "stamps read")
    seg = [out[0], out[1], out[2]]
    tot = sum(seg)
    waves = out[3]
    ksteps = waves * (n // 64)
    print("RESULT " + json.dumps({
        "size": n, "variant": variant, "waves": waves,
        "share_kstep0": round(seg[0] / tot, 4), "share_wait_barrier": round(seg[1] / tot, 4),
        "share_kstep1": round(seg[2] / tot, 4),
        "cycles_per_kiter": {"kstep0": round(seg[0] / ksteps, 1), "wait_barrier": round(seg[1] / ksteps, 1),
                             "kstep1": round(seg[2] / ksteps, 1)},
        "note": "s_memtime ticks; 64 MFMAs per k-step = 1024 cycles at issue rate"}))


if __name__ == "__main__":
    main()
