#!/usr/bin/env python3
"""Locate wrong output blocks of one GEMM schedule variant (debug aid).

    python scripts/gpu/gemm_variant_debug.py VARIANT
For each (M, N, K) prints the max error and which 16x16 blocks / waves are
wrong, so a schedule race can be pinned to an operand region and K-tile."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxk8s.ops import _lib  # noqa: E402


def main():
    v = int(sys.argv[1])
    L = _lib.lib()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    for (M, N, K) in [(256, 256, 64), (256, 256, 128), (256, 256, 192), (256, 256, 256),
                      (256, 256, 512), (512, 512, 1024), (4096, 4096, 256)]:
        a = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).bfloat16()
        b = (torch.rand(N, K, device=dev, generator=g) * 2 - 1).bfloat16()
        c = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
        st = L.mxk_gemm_bf16_tn_variant(a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, K, K, N,
                                        v, _lib.stream_ptr(dev))
        _lib.check(st, "variant")
        torch.cuda.synchronize()
        ref = a.float() @ b.float().t()
        err = (c.float() - ref).abs()
        blk = err.view(M // 16, 16, N // 16, 16).amax(dim=(1, 3))
        bad = (blk > 0.05 * K ** 0.5).nonzero().tolist()
        # which k-stage's contribution is missing/wrong: project the error on each 64-k slice
        d = (c.float() - ref)
        k_corr = []
        for s in range(K // 64):
            part = a[:, s * 64:(s + 1) * 64].float() @ b[:, s * 64:(s + 1) * 64].float().t()
            k_corr.append(round(float((d * part).sum() / (part * part).sum()), 3))
        print(f"M={M} N={N} K={K} max_err={err.max().item():.3f} bad_blocks={len(bad)}/{blk.numel()} "
              f"first={bad[:6]} stage_coeff={k_corr[:12]}", flush=True)


if __name__ == "__main__":
    main()
