#!/usr/bin/env python3
"""Group a rocprofv3 ``--stats`` kernel CSV into op categories (ms per step).

    python scripts/kernel_breakdown.py <kernel_stats.csv> --steps N
"""
import argparse
import csv
import re

CATS = [
    ("gemm.hipblaslt", r"^Cijk_|^Custom_Cijk"),
    ("gemm.mxk_wgrad", r"mxk_gemm_bf16_x_kernel"),
    ("gemm.mxk", r"mxk_gemm_bf16"),
    ("attn.fwd", r"mxk_attn_fwd"),
    ("attn.bwd", r"mxk_attn_bwd"),
    ("adamw", r"adamw"),
    ("grad_norm", r"sumsq|fold_sum|scale_from"),
    ("rmsnorm", r"rmsnorm"),
    ("swiglu", r"swiglu"),
    ("rope", r"rope"),
    ("xent", r"xent"),
    ("rccl", r"nccl|rccl"),
    ("copy/fill", r"copy|fill|memset|Memcpy|elementwise|reduce|embedding|index"),
]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("csv")
    p.add_argument("--steps", type=int, required=True)
    a = p.parse_args()
    tot = {}
    names = {}
    with open(a.csv) as f:
        for row in csv.DictReader(f):
            name, ns = row["Name"], float(row["TotalDurationNs"])
            cat = next((c for c, rx in CATS if re.search(rx, name)), "other")
            tot[cat] = tot.get(cat, 0.0) + ns
            names.setdefault(cat, []).append((ns, name[:90]))
    allns = sum(tot.values())
    print(f"{'category':18s} {'ms/step':>9s} {'share':>7s}")
    for cat, ns in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"{cat:18s} {ns / 1e6 / a.steps:9.2f} {ns / allns:7.1%}")
    print(f"{'total':18s} {allns / 1e6 / a.steps:9.2f}")
    print("\ntop kernels of 'other' and 'copy/fill':")
    for cat in ("other", "copy/fill"):
        for ns, n in sorted(names.get(cat, []), reverse=True)[:6]:
            print(f"  {cat:10s} {ns / 1e6 / a.steps:8.2f}  {n}")


if __name__ == "__main__":
    main()
