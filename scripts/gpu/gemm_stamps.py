#!/usr/bin/env python3
"""Where a K-tile of the default GEMM schedule spends its cycles: runs the
stamped diagnostic build of schedule 26 (experiments library, schedule 45)
after a >= 2 s warm-up on random data and prints, per shape, the mean shader
cycles per DMA-carrying K-tile of each wave in

  wait1   s_waitcnt lgkmcnt(0) + barrier #1 (A k-half-1 fragment reads)
  wait2   s_waitcnt lgkmcnt(0) + barrier #2 (B k-half-1 fragment reads)
  wait3   counted vmcnt (stage s+1 landed) + barrier #3
  period  barrier #3 -> barrier #3 (the whole K-tile)

against the 128 x 16 = 2048-cycle MFMA floor of a K-tile, and the quantiles
over waves.  The stamps (s_memtime, an SMEM round trip each) add cycles of
their own: compare waits with each other, not with the production kernel.

    MXK_KERNELS_LIB=mxk8s/_lib/libmxkernels_exp.so python scripts/gpu/gemm_stamps.py
"""
import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mxk8s.ops import _lib  # noqa: E402


def main() -> int:
    L = _lib.lib()
    if not hasattr(L, "mxk_gemm_stamps_read") or not L.mxk_gemm_bf16_tn_variant_built(45):
        raise SystemExit("needs the experiments library (MXK_KERNELS_LIB=...libmxkernels_exp.so)")
    dev = torch.device("cuda", 0)
    shapes = [tuple(int(v) for v in s.split("x"))
              for s in os.environ.get("SHAPES", "8192x8192x8192,4096x4096x16384,4096x4096x4096").split(",")]
    for M, N, K in shapes:
        g = torch.Generator(device=dev)
        g.manual_seed(1)
        A = (torch.rand((M, K), device=dev, generator=g) * 2 - 1).bfloat16()
        Bt = (torch.rand((N, K), device=dev, generator=g) * 2 - 1).bfloat16()
        C = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        st = _lib.stream_ptr(dev)

        def run(v):
            _lib.check(L.mxk_gemm_bf16_tn_variant(A.data_ptr(), Bt.data_ptr(), C.data_ptr(), M, N, K,
                                                  K, K, N, v, st), f"variant {v}")
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 2.0:
            for _ in range(10):
                run(26)
            torch.cuda.synchronize()
        for _ in range(3):
            run(45)
        torch.cuda.synchronize()
        ref = torch.matmul(A, Bt.t())
        ok = ((C.float() - ref.float()).norm() / ref.float().norm()).item() < 1e-2
        nwaves = (M // 256) * (N // 256) * 4
        buf = (ctypes.c_ulonglong * (nwaves * 8))()
        _lib.check(L.mxk_gemm_stamps_read(ctypes.cast(buf, ctypes.c_void_p), nwaves * 8), "stamps")
        rows = [list(buf[i * 8:(i + 1) * 8]) for i in range(nwaves)]
        per = {k: [] for k in ("wait1", "wait2", "wait3", "period", "loop_per_ktile")}
        for r in rows:
            n = max(1, r[4])
            per["wait1"].append(r[0] / n)
            per["wait2"].append(r[1] / n)
            per["wait3"].append(r[2] / n)
            per["period"].append(r[3] / max(1, n - 1))
            per["loop_per_ktile"].append(r[5] / (K // 64))
        out = {"M": M, "N": N, "K": K, "check_ok": ok, "waves": nwaves, "mfma_floor": 2048}
        for k, v in per.items():
            v = sorted(v)
            out[k] = {"mean": round(sum(v) / len(v), 1), "p10": round(v[len(v) // 10], 1),
                      "p50": round(v[len(v) // 2], 1), "p90": round(v[9 * len(v) // 10], 1)}
        # wave-to-wave skew inside a workgroup: spread of loop start stamps
        starts = [r[6] for r in rows]
        skew = [max(starts[i:i + 4]) - min(starts[i:i + 4]) for i in range(0, len(starts), 4)]
        out["start_skew_in_wg_p50"] = sorted(skew)[len(skew) // 2]
        print("RESULT " + json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
