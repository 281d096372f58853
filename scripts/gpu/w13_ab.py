#!/usr/bin/env python3
"""Fused up-projection + SwiGLU (mxk_gemm_bf16_w13_swiglu) at the Llama-3-8B
step shape (16384 tokens, F 14336, K 4096): K-loop schedules 0 (production),
1 (one-barrier loop) and 3 (persistent) from the experiments library,
interleaved rounds, median ms and TF/s; outputs checked equal to schedule 0
(schedule 3 runs the same K loop as 1: bit-identical to it)."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxk8s.ops import _lib  # noqa: E402
from mxk8s.ops.linear import w13_swiglu  # noqa: E402

M, F, K = int(os.environ.get("M", 16384)), 14336, 4096
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
x = (torch.randn((M, K), device=dev, generator=g) * 0.5).bfloat16()
w = (torch.randn((2 * F, K), device=dev, generator=g) * K ** -0.5).bfloat16()
L = _lib.lib()
scheds = [int(v) for v in os.environ.get("SCHEDS", "0,1,3").split(",")]
outs = {}
for s in scheds:
    L.mxk_gemm_w13_set_sched(s)
    outs[s] = w13_swiglu(x, w)
torch.cuda.synchronize()
for s in scheds[1:]:
    same = all(torch.equal(a, b) for a, b in zip(outs[scheds[0]], outs[s]))
    print(f"RESULT sched={s} equal to sched={scheds[0]}: {same}", flush=True)
if 1 in outs and 3 in outs:
    print("RESULT sched=3 equal to sched=1:", all(torch.equal(a, b) for a, b in zip(outs[1], outs[3])), flush=True)
ts = {s: [] for s in scheds}
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
for _ in range(8):
    for s in scheds:
        L.mxk_gemm_w13_set_sched(s)
        for _ in range(2):
            w13_swiglu(x, w)
        ev[0].record()
        for _ in range(10):
            w13_swiglu(x, w)
        ev[1].record()
        torch.cuda.synchronize()
        ts[s].append(ev[0].elapsed_time(ev[1]) / 10)
L.mxk_gemm_w13_set_sched(0)
for s in scheds:
    ms = statistics.median(ts[s])
    print(f"RESULT w13 sched={s} M={M} ms={ms:.4f} tflops={2 * M * 2 * F * K / ms / 1e9:.1f}", flush=True)
