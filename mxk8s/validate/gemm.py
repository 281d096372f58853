"""Validator config 3: CDNA4 bf16 MFMA GEMM throughput + correctness.

Protocol (BASELINE.md "Measurement protocol"): random uniform [-1, 1) bf16
operands (never zeros: DVFS clocks higher on zeros), >= 2 s of warm-up
launches, then the median of >= 50 timed launches with HIP events;
TFLOPS = 2*M*N*K / t.  Correctness: fp32 reference on a sub-block and
relative error against hipBLASLt (torch.matmul) on the full output.

Schedules of the 256x256 kernel are A/B-timed in ONE process with rounds
interleaved (cdna_hip_programming.md §5.4 rule 24) when --variants is given.

    python -m mxk8s.validate.gemm --sizes 4096,8192,16384 [--variants all]

The production library carries the shipped schedules only; the A/B records
(schedules measured neutral or negative, the no-store ablation) are in
``make gemm-exp``'s libmxkernels_exp.so, selected with
``MXK_KERNELS_LIB=mxk8s/_lib/libmxkernels_exp.so``.

Prints one ``RESULT {json}`` line per (size, kernel).
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time

import torch

from ..ops import _lib
from ..ops.gemm import gemm_bf16_tn
from ..utils import roctx


def _events_time(fn, iters: int) -> list[float]:
    """Seconds per launch over one block of ``iters`` back-to-back launches.

    (Until round 2 each launch was timed alone with a synchronize after it:
    every kernel then started on an idle GPU, which at 4096^3 (~0.1 ms)
    costs hipBLASLt ~13 % and this kernel ~3 %, and made the hand-written
    kernel look 9-10 % ahead there; back to back it is 3 % behind.)"""
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return [s.elapsed_time(e) * 1e-3 / iters]


def run(sizes, variants, iters: int, warmup_s: float, rounds: int, device=None,
        is_ablation=lambda v: False, pad: int = 0, cold: int = 1) -> list[dict]:
    dev = device or torch.device("cuda", torch.cuda.current_device())
    L = _lib.lib()
    stream = lambda: _lib.stream_ptr(dev)  # noqa: E731
    results = []
    for n in sizes:
        M, N, K = n if isinstance(n, tuple) else (n, n, n)
        g = torch.Generator(device=dev)
        g.manual_seed(M * 7 + N * 3 + K)
        # pad > 0: operands are [:, :K] views of (rows, K + pad) buffers, so
        # lda = ldb = K + pad (a diagnostic of power-of-two row strides)
        # cold > 1: that many operand pairs, each launch takes the next one, so
        # with cold x (A + B) beyond the 256 MB Infinity Cache every launch
        # streams its operands from HBM as in a training step (back-to-back
        # launches of one pair run from the cache)
        pairs = [((torch.rand((M, K + pad), device=dev, generator=g) * 2 - 1).bfloat16()[:, :K],
                  (torch.rand((N, K + pad), device=dev, generator=g) * 2 - 1).bfloat16()[:, :K])
                 for _ in range(max(1, cold))]
        A, Bt = pairs[0]
        lda = ldb = K + pad
        C = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
        ref = torch.matmul(A, Bt.t())
        kernels = {}
        turn = [0]

        def nxt():
            turn[0] += 1
            return pairs[turn[0] % len(pairs)]
        for v in variants:
            def mk(v=v):
                a, b = nxt()
                st = L.mxk_gemm_bf16_tn_variant(a.data_ptr(), b.data_ptr(), C.data_ptr(), M, N, K,
                                                lda, ldb, N, v, stream())
                if st:
                    _lib.check(st, f"gemm variant {v}")
            name = L.mxk_gemm_bf16_tn_variant_name(v)
            kernels[f"mxk_v{v}_{name.decode() if name else '?'}"] = mk

        def default():
            a, b = nxt()
            gemm_bf16_tn(a, b, C)

        def lib():
            a, b = nxt()
            torch.matmul(a, b.t(), out=C)
        kernels["mxk_default"] = default
        kernels["hipblaslt"] = lib
        # correctness of every hand-written schedule
        checks = {}
        ablations = set(k for k in kernels if k.startswith("mxk_v") and
                        is_ablation(int(k[5:].split("_")[0])))
        for name, fn in kernels.items():
            if name == "hipblaslt" or name in ablations:
                continue
            C.zero_()
            turn[0] = len(pairs) - 1          # the next launch takes pair 0
            fn()
            torch.cuda.synchronize()
            rel = ((C.float() - ref.float()).norm() / ref.float().norm()).item()
            sub = (A[:128].float() @ Bt[:128].float().t())
            sub_err = (C[:128, :128].float() - sub).abs().max().item()
            checks[name] = (rel, sub_err)
            if not (rel < 1e-2 and sub_err <= 2 ** -7 * sub.abs().max().item() + 1e-3):
                raise RuntimeError(f"{name} wrong at {n}: rel {rel}, max sub err {sub_err}")
        # warm up >= warmup_s on random data (clock settles under load)
        t0 = time.perf_counter()
        with roctx.range(f"gemm.warmup.{n}"):
            while time.perf_counter() - t0 < warmup_s:
                for fn in kernels.values():
                    fn()
                torch.cuda.synchronize()
        samples = {k: [] for k in kernels}
        for _ in range(rounds):
            for name, fn in kernels.items():
                with roctx.range(f"gemm.timed.{name}.{n}"):
                    samples[name] += _events_time(fn, max(1, iters // rounds))
        flops = 2.0 * M * N * K
        for name, ts in samples.items():
            med = statistics.median(ts)
            r = {"kernel": name, "M": M, "N": N, "K": K, "lda": lda, "dtype": "bf16",
                 "median_ms": med * 1e3, "min_ms": min(ts) * 1e3,
                 "tflops_median": flops / med / 1e12, "tflops_best": flops / min(ts) / 1e12,
                 "samples": len(ts), "data": "uniform[-1,1) random", "cold_pairs": len(pairs)}
            if name in checks:
                r["rel_err_vs_hipblaslt"], r["max_abs_err_subblock_vs_fp32"] = checks[name]
            results.append(r)
            print("RESULT " + json.dumps(r), flush=True)
    return results


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--sizes", default="4096,8192,16384")
    p.add_argument("--shapes", default="", help="extra MxNxK shapes, comma separated")
    p.add_argument("--variants", default="", help="'all' or comma list of schedule ids")
    p.add_argument("--iters", type=int, default=60)
    p.add_argument("--rounds", type=int, default=6)
    p.add_argument("--warmup-s", type=float, default=2.0)
    p.add_argument("--device", type=int, default=None)
    p.add_argument("--pad", type=int, default=0, help="lda = ldb = K + pad (multiple of 8)")
    p.add_argument("--cold", type=int, default=1,
                   help="operand pairs cycled per launch (beyond the Infinity Cache: HBM-cold)")
    a = p.parse_args(argv)
    if a.device is not None:
        torch.cuda.set_device(a.device)
    L = _lib.lib()
    nv = L.mxk_gemm_bf16_tn_num_variants()
    if a.variants == "all":
        variants = [v for v in range(nv) if L.mxk_gemm_bf16_tn_variant_built(v)]
    elif a.variants:
        variants = [int(x) for x in a.variants.split(",")]
    else:
        variants = []
    missing = [v for v in variants if not L.mxk_gemm_bf16_tn_variant_built(v)]
    if missing:
        raise SystemExit(f"schedules {missing} are A/B records, not in {_lib.KERNEL_LIB_PATH}: "
                         "`make gemm-exp` and run with "
                         "MXK_KERNELS_LIB=mxk8s/_lib/libmxkernels_exp.so")
    sizes = [int(x) for x in a.sizes.split(",")] if a.sizes else []
    sizes += [tuple(int(v) for v in x.split("x")) for x in a.shapes.split(",") if x]
    run(sizes, variants, a.iters, a.warmup_s, a.rounds,
        is_ablation=lambda v: bool(_lib.lib().mxk_gemm_bf16_tn_is_ablation(v)), pad=a.pad,
        cold=a.cold)
    return 0


if __name__ == "__main__":
    sys.exit(main())
