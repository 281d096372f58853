#!/usr/bin/env python3
"""Tune (PyTorch TunableOp: every hipBLASLt + rocBLAS solution) the 15 GEMMs
of a Llama-3-8B training step — forward, dgrad and wgrad of the five linear
layer shapes at T tokens — and write the winning-solution table that the
trainer loads read-only (mxk8s/train/tunableop_mi355x.csv).

    PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 \
    PYTORCH_TUNABLEOP_FILENAME=out.csv python scripts/tune_gemms.py --tokens 8192

With --bench (tuning off) it times each GEMM and prints RESULT lines.
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

SHAPES = [(4096, 6144, "wqkv"), (4096, 4096, "wo"), (4096, 28672, "w13"), (14336, 4096, "w2"),
          (4096, 128256, "lm_head")]


def ops(T, din, dout, dev):
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(T, din, device=dev, generator=g).bfloat16()
    w = torch.randn(dout, din, device=dev, generator=g).bfloat16() * 0.02
    dy = torch.randn(T, dout, device=dev, generator=g).bfloat16()
    dw = torch.empty(dout, din, device=dev, dtype=torch.bfloat16)
    return {
        "fwd": lambda: torch.matmul(x, w.t()),
        "dgrad": lambda: torch.matmul(dy, w),
        "wgrad": lambda: torch.matmul(dy.t(), x, out=dw),
    }


def timeit(fn, iters=20):
    for _ in range(3):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--bench", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    for din, dout, name in SHAPES:
        for kind, fn in ops(a.tokens, din, dout, dev).items():
            t0 = time.time()
            fn()
            torch.cuda.synchronize()
            rec = {"gemm": f"{name}.{kind}", "T": a.tokens, "in": din, "out": dout,
                   "first_call_s": round(time.time() - t0, 1)}
            if a.bench:
                ms = timeit(fn)
                rec.update(ms=round(ms, 4), tflops=round(2 * a.tokens * din * dout / ms / 1e9, 1))
            print("RESULT " + json.dumps(rec), flush=True)
    # TunableOp writes PYTORCH_TUNABLEOP_FILENAME when the process exits


if __name__ == "__main__":
    sys.exit(main())
