#!/usr/bin/env python3
"""The Llama-3-8B step's GEMM products, isolated, against hipBLASLt on the
same operands and layouts (is the step's rate a property of
the kernels or of the shapes?).

Tokens T = 16384 (micro-batch 8 x seq 2048).  Per product:
  fwd    Y[T,N]  = X[T,K] . W[N,K]^T   mxk: gemm_bf16_tn        torch: x @ w.t()
  dgrad  dX[T,K] = dY[T,N] . W[N,K]    mxk: gemm_bf16_ex(K-major A, N-major B)  torch: dy @ w
  wgrad  dW[N,K] = dY[T,N]^T . X[T,K]  mxk: gemm_bf16_ex(M-major A, N-major B)  torch: dy.t() @ x
Plain products only (the SwiGLU epilogues are priced in
profiles/r4_step/swiglu_epilogue_price.log).  Uniform random bf16 operands,
warm; the two kernels alternate over --rounds rounds of --iters launches and
the medians are compared.  Prints one RESULT json line per product.
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxk8s.ops import gemm as G  # noqa: E402

T, D, F, QKV = 16384, 4096, 14336, 6144
PRODUCTS = [   # name, kind, N (output features), K (input features)
    ("wqkv.fwd", "fwd", QKV, D), ("wo.fwd", "fwd", D, D), ("w13.fwd", "fwd", 2 * F, D),
    ("w2.fwd", "fwd", D, F),
    ("wqkv.dgrad", "dgrad", QKV, D), ("wo.dgrad", "dgrad", D, D), ("w13.dgrad", "dgrad", 2 * F, D),
    ("w2.dgrad", "dgrad", D, F),
    ("wqkv.wgrad", "wgrad", QKV, D), ("wo.wgrad", "wgrad", D, D), ("w13.wgrad", "wgrad", 2 * F, D),
    ("w2.wgrad", "wgrad", D, F),
]


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--only", default="", help="comma list of product names")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*shape):
        return (torch.rand(*shape, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)

    only = set(a.only.split(",")) if a.only else None
    for name, kind, N, K in PRODUCTS:
        if only and name not in only:
            continue
        w = rnd(N, K)
        if kind == "fwd":
            x = rnd(T, K)
            out = torch.empty(T, N, device=dev, dtype=torch.bfloat16)
            mxk = lambda: G.gemm_bf16_tn(x, w, out=out)   # noqa: E731
            lib = lambda: torch.matmul(x, w.t())          # noqa: E731
            ref = lambda: x.float() @ w.float().t()       # noqa: E731
        elif kind == "dgrad":
            dy = rnd(T, N)
            out = torch.empty(T, K, device=dev, dtype=torch.bfloat16)
            mxk = lambda: G.gemm_bf16_ex(dy, w, True, False, out)   # noqa: E731
            lib = lambda: torch.matmul(dy, w)                       # noqa: E731
            ref = lambda: dy.float() @ w.float()                    # noqa: E731
        else:
            dy, x = rnd(T, N), rnd(T, K)
            out = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
            mxk = lambda: G.gemm_bf16_ex(dy, x, False, False, out)   # noqa: E731
            lib = lambda: torch.matmul(dy.t(), x)                    # noqa: E731
            ref = lambda: dy.float().t() @ x.float()                 # noqa: E731
        assert mxk() is not False, f"{name}: shape not taken by the mxk kernel"
        torch.cuda.synchronize()
        r = ref()
        err = (out.float() - r).abs().max().item()
        tol = 0.02 * r.abs().max().item() + 0.5
        del r
        flops = 2.0 * T * N * K
        for _ in range(3):
            mxk()
            lib()
        tm, tl = [], []
        for _ in range(a.rounds):
            tm.append(timed(mxk, a.iters))
            tl.append(timed(lib, a.iters))
        m, l = statistics.median(tm), statistics.median(tl)
        print("RESULT " + json.dumps({
            "product": name, "MNK": {"fwd": (T, N, K), "dgrad": (T, K, N), "wgrad": (N, K, T)}[kind],
            "mxk_ms": round(m, 4), "hipblaslt_ms": round(l, 4),
            "mxk_tflops": round(flops / m / 1e9, 1), "hipblaslt_tflops": round(flops / l / 1e9, 1),
            "mxk_over_hipblaslt": round(l / m, 4), "max_err": round(err, 3), "ok": err <= tol}),
            flush=True)
        del w, out
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
