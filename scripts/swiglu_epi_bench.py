#!/usr/bin/env python3
"""Price the dgrad-SwiGLU GEMM's epilogue (Llama-3-8B down projection at 16k
tokens: dh = dy W2, M 16384, F 14336, K 4096) by timing, back to back and
interleaved over rounds, in one process:

  plain    the same GEMM with a plain LDS-staged bf16 store of dh (x2 dgrad)
  epi4     the production fused epilogue (g/u of pass 0 prefetched)
  epi5     epi4 without the prefetch
  epi6     epi4 without the SwiGLU math (same memory traffic; wrong values)
  epi3     the permlane-pair epilogue
  epi8     epi4 with the rounds staggered by XCD group

(modes 5, 6 and 8 are A/B records: run with
MXK_KERNELS_LIB=mxk8s/_lib/libmxkernels_exp.so, or they time the default)

Prints one RESULT json per kernel (median ms, TF/s of the GEMM part)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxk8s.ops import _lib, gemm  # noqa: E402


def main() -> int:
    dev = torch.device("cuda", 0)
    M, F, K = 16384, 14336, 4096
    g = torch.Generator(device=dev).manual_seed(3)
    dy = (torch.randn((M, K), device=dev, generator=g) * 0.5).bfloat16()
    w2 = (torch.randn((K, F), device=dev, generator=g) * K ** -0.5).bfloat16()
    gu = (torch.randn((M, 2 * F), device=dev, generator=g) * 2).bfloat16()
    dgu = torch.empty_like(gu)
    dh = torch.empty((M, F), device=dev, dtype=torch.bfloat16)
    L = _lib.lib()
    st = _lib.stream_ptr(dev)

    def fused(mode):
        def f():
            L.mxk_gemm_swiglu_set_epi(mode)
            _lib.check(L.mxk_gemm_bf16_dgrad_swiglu(dy.data_ptr(), w2.data_ptr(), gu.data_ptr(),
                                                    dgu.data_ptr(), M, F, K, K, F, st), "dgrad_swiglu")
        return f

    kernels = {"plain": lambda: gemm.gemm_bf16_ex(dy, w2, True, False, dh),
               "epi4": fused(4), "epi5": fused(5), "epi6": fused(6), "epi3": fused(3),
               "epi8": fused(8)}
    for fn in kernels.values():
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    ts = {k: [] for k in kernels}
    for _ in range(int(os.environ.get("ROUNDS", 8))):
        for name, fn in kernels.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(10):
                fn()
            e.record()
            e.synchronize()
            ts[name].append(s.elapsed_time(e) / 10)
    L.mxk_gemm_swiglu_set_epi(4)
    flops = 2.0 * M * F * K
    for name, v in ts.items():
        m = statistics.median(v)
        print("RESULT " + json.dumps({"kernel": name, "ms": round(m, 4),
                                      "tflops": round(flops / m / 1e9, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
