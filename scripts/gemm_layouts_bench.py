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


def timeit(fns, iters=30, rounds=6):
    """Median seconds-per-launch of each fn over A/B-interleaved blocks of
    back-to-back launches (one event pair per block: a synchronize after
    every launch starts each kernel on an idle GPU and biases small and
    medium GEMMs, hipBLASLt's more than this kernel's)."""
    for f in fns:
        for _ in range(5):
            f()
    torch.cuda.synchronize()
    ts = [[] for _ in fns]
    for r in range(rounds):
        order = list(range(len(fns)))
        if r % 2:
            order.reverse()
        for i in order:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(iters):
                fns[i]()
            e.record()
            e.synchronize()
            ts[i].append(s.elapsed_time(e) / iters)
    return [statistics.median(t) for t in ts]


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
            fns, names = [], []
            for v in VARIANTS:
                out.zero_()
                ok = gemm_bf16_ex(a, b, ak, bk, out, variant=v)
                if not ok:
                    res[f"mxk_v{v}_tflops"] = None
                    continue
                rel = ((out.float() - ref.float()).norm() / ref.float().norm()).item()
                if not rel < 1e-2:
                    raise SystemExit(f"{name}.{kind} variant {v}: wrong result rel {rel}")
                fns.append(lambda v=v: gemm_bf16_ex(a, b, ak, bk, out, variant=v))
                names.append(f"mxk_v{v}_tflops")
            out2 = torch.empty(shp, device=dev, dtype=torch.bfloat16)
            blas = {"fwd": lambda: torch.matmul(x, w.t(), out=out2),
                    "dgrad": lambda: torch.matmul(dy, w, out=out2),
                    "wgrad": lambda: torch.matmul(dy.t(), x, out=out2)}[kind]
            fns.append(blas)
            names.append("hipblaslt_tflops")
            for nm, t in zip(names, timeit(fns)):
                res[nm] = round(flops / t / 1e9, 1)
            print("RESULT " + json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
