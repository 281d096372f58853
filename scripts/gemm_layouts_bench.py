#!/usr/bin/env python3
"""Correctness + TFLOPS of the layout-generic MFMA GEMM vs hipBLASLt
(torch.matmul) on the Llama-3-8B training-step GEMMs (fwd / dgrad / wgrad)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxk8s.ops.gemm import gemm_bf16_ex  # noqa: E402

VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "1").split(",")]
SHAPES = [(4096, 6144, "wqkv"), (4096, 4096, "wo"), (4096, 28672, "w13"), (14336, 4096, "w2")]


def timeit(fn, iters=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


def main():
    T = int(os.environ.get("TOKENS", 8192))
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for din, dout, name in SHAPES:
        x = (torch.rand(T, din, device=dev, generator=g) * 2 - 1).bfloat16()
        w = (torch.rand(dout, din, device=dev, generator=g) * 2 - 1).bfloat16()
        dy = (torch.rand(T, dout, device=dev, generator=g) * 2 - 1).bfloat16()
        cases = {
            "fwd": (x, w, True, True, (T, dout), lambda: torch.matmul(x, w.t())),
            "dgrad": (dy, w, True, False, (T, din), lambda: torch.matmul(dy, w)),
            "wgrad": (dy, x, False, False, (dout, din), lambda: torch.matmul(dy.t(), x)),
        }
        for kind, (a, b, ak, bk, shp, ref_fn) in cases.items():
            out = torch.empty(shp, device=dev, dtype=torch.bfloat16)
            ref = ref_fn()
            K = din if kind == "fwd" else (dout if kind == "dgrad" else T)
            flops = 2.0 * shp[0] * shp[1] * K
            res = {"gemm": f"{name}.{kind}", "M": shp[0], "N": shp[1], "K": K}
            for v in VARIANTS:
                out.zero_()
                ok = gemm_bf16_ex(a, b, ak, bk, out, variant=v)
                if not ok:
                    res[f"mxk_v{v}_tflops"] = None
                    continue
                rel = ((out.float() - ref.float()).norm() / ref.float().norm()).item()
                if not rel < 1e-2:
                    raise SystemExit(f"{name}.{kind} variant {v}: wrong result rel {rel}")
                t = timeit(lambda: gemm_bf16_ex(a, b, ak, bk, out, variant=v))
                res[f"mxk_v{v}_tflops"] = round(flops / t / 1e9, 1)
            res["hipblaslt_tflops"] = round(flops / timeit(ref_fn) / 1e9, 1)
            print("RESULT " + json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
