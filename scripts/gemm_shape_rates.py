#!/usr/bin/env python3
"""Per-shape TFLOP/s of the Llama-3-8B step GEMMs from a rocprofv3 kernel
trace of ``bench.py --mode ddp`` (16k tokens: B 8 x S 2048).  Dispatches are
keyed by kernel template and grid; products that share a kernel and grid are
told apart by duration band (K differs).

    python scripts/gemm_shape_rates.py <kernel_trace.csv> [--steps N]
"""
import argparse
import csv
import statistics

T, D, F, QKV, V = 16384, 4096, 14336, 6144, 128256
# (kernel substring, grid threads, duration band ms): (name, flops)
SHAPES = {
    ("tn_w4", 262144, 0.25, 0.8): ("wo.fwd", 2 * T * D * D),
    ("tn_w4", 262144, 0.8, 2.0): ("w2.fwd", 2 * T * D * F),
    ("tn_w4", 393216, 0.0, 9.0): ("wqkv.fwd", 2 * T * QKV * D),
    ("w13_swiglu", 1835008, 0.0, 9.0): ("w13.fwd+swiglu", 2 * T * 2 * F * D),
    ("x2_kernel<false, true, 1, 0, false>", 262144, 0.25, 0.48): ("wo.dgrad", 2 * T * D * D),
    ("x2_kernel<false, true, 1, 0, false>", 262144, 0.48, 0.8): ("wqkv.dgrad", 2 * T * D * QKV),
    ("x2_kernel<false, true, 1, 0, false>", 262144, 2.0, 3.5): ("w13.dgrad", 2 * T * D * 2 * F),
    ("x2_kernel<false, true, 1, 0, false>", 262144, 9.0, 20.0): ("lm.dgrad", 2 * T * D * V),
    ("x2_kernel<false, true, 4, 0, false>", 917504, 0.0, 9.0): ("w2.dgrad+swiglu", 2 * T * F * D),
    ("x2_kernel<true, true, 1, 1, false>", 458752, 0.0, 9.0): ("w13.wgrad", 2 * T * D * 2 * F),
    ("x2_kernel<true, true, 1, 1, false>", 65536, 0.0, 9.0): ("wo.wgrad (+wqkv main)", 2 * T * D * D),
}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("trace")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    print(f"{'product':26s} {'n':>5s} {'median ms':>10s} {'TF/s':>8s}")
    for (pat, grid, lo, hi), (name, flops) in SHAPES.items():
        v = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows
             if pat in r["Kernel_Name"] and int(r["Grid_Size_X"]) == grid]
        v = [x for x in v if lo <= x < hi]
        if not v:
            continue
        m = statistics.median(v)
        print(f"{name:26s} {len(v):5d} {m:10.4f} {flops / m / 1e9:8.1f}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
