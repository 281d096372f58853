#!/usr/bin/env python3
"""Run the MFMA GEMM in each operand layout on one shape (for rocprofv3
counter passes comparing the TN kernel with the layout kernel):
    tn  A [M][K], B [N][K]   (mxk_gemm_bf16_tn)
    tnx the same operands on the layout kernel (x2, K-major both)
    mix A [M][K], B [K][N]   (dgrad: x2 kernel, B transposed reads)
    nn  A [K][M], B [K][N]   (wgrad: x2 kernel, both transposed reads)
Prints TFLOPS per layout (CUDA-event timed) after the counted iterations."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxk8s.ops.gemm import gemm_bf16_ex  # noqa: E402

M, N, K = (int(x) for x in os.environ.get("SHAPE", "8192x8192x8192").split("x"))
ITERS = int(os.environ.get("ITERS", "20"))
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
r = lambda *s: (torch.rand(*s, device=dev, generator=g) * 2 - 1).bfloat16()  # noqa: E731
a_k, a_m, b_k, b_n = r(M, K), r(K, M), r(N, K), r(K, N)
out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
cases = {"tn": (a_k, b_k, True, True, 1), "tnx": (a_k, b_k, True, True, 2),
         "mix": (a_k, b_n, True, False, 1), "nn": (a_m, b_n, False, False, 1)}
for name in os.environ.get("LAYOUTS", "tn,tnx,mix,nn").split(","):
    a, b, ak, bk, var = cases[name]
    ts = []
    for _ in range(ITERS):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        assert gemm_bf16_ex(a, b, ak, bk, out, variant=var)
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    t = statistics.median(ts[2:])
    print(f"{name} {M}x{N}x{K}: {2.0 * M * N * K / t / 1e9:.1f} TF/s ({t:.3f} ms)", flush=True)
