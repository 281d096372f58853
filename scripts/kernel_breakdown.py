#!/usr/bin/env python3
"""Group rocprofv3 kernel times into op categories (ms per step).

Steady state only (default, from a kernel TRACE):

    python scripts/kernel_breakdown.py --trace <kernel_trace.csv> \
        --markers <marker_api_trace.csv> --range bench.timed --steps N

keeps the dispatches that START inside the ``bench.timed`` roctx range the
trainer pushes around its timed steps (``mxk8s/train/ddp_llama.py``), so
initialisation and warm-up kernels (a 83 ms one-time bf16->fp32 master copy
was counted per step in round 2) are out, and also prints the range's own
wall time per step: the category sum is then checkable against it (kernels
of one stream; RCCL on its own stream may overlap and add to the sum).

Whole-run totals (``--stats`` CSV, every kernel of the process):

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


def category(name: str) -> str:
    return next((c for c, rx in CATS if re.search(rx, name)), "other")


def _col(row: dict, *cands):
    for c in cands:
        if c in row:
            return row[c]
    for k in row:                      # tolerate spelling differences between versions
        if any(c.lower() in k.lower() for c in cands):
            return row[k]
    raise KeyError(cands)


def window(markers_csv: str, name: str) -> tuple[int, int]:
    """[start, end] ns of the (first) roctx range called ``name``."""
    with open(markers_csv) as f:
        for row in csv.DictReader(f):
            label = " ".join(str(v) for v in row.values())
            if name in label:
                return int(_col(row, "Start_Timestamp")), int(_col(row, "End_Timestamp"))
    raise SystemExit(f"no roctx range {name!r} in {markers_csv}")


def from_trace(trace_csv: str, lo: int, hi: int) -> list[tuple[str, float]]:
    out = []
    with open(trace_csv) as f:
        for row in csv.DictReader(f):
            t0, t1 = int(_col(row, "Start_Timestamp")), int(_col(row, "End_Timestamp"))
            if lo <= t0 <= hi:
                out.append((_col(row, "Kernel_Name", "Name"), float(t1 - t0)))
    return out


def from_stats(stats_csv: str) -> list[tuple[str, float]]:
    with open(stats_csv) as f:
        return [(row["Name"], float(row["TotalDurationNs"])) for row in csv.DictReader(f)]


def breakdown(rows, steps: int, wall_ns: float | None = None) -> str:
    tot, names = {}, {}
    for name, ns in rows:
        cat = category(name)
        tot[cat] = tot.get(cat, 0.0) + ns
        names.setdefault(cat, {}).setdefault(name[:90], 0.0)
        names[cat][name[:90]] += ns
    allns = sum(tot.values()) or 1.0
    out = [f"{'category':18s} {'ms/step':>9s} {'share':>7s}"]
    for cat, ns in sorted(tot.items(), key=lambda kv: -kv[1]):
        out.append(f"{cat:18s} {ns / 1e6 / steps:9.2f} {ns / allns:7.1%}")
    out.append(f"{'total':18s} {allns / 1e6 / steps:9.2f}")
    if wall_ns is not None:
        out.append(f"{'range wall':18s} {wall_ns / 1e6 / steps:9.2f}   "
                   f"(kernel sum / wall = {allns / wall_ns:.3f})")
    out.append("\ntop kernels of 'other' and 'copy/fill':")
    for cat in ("other", "copy/fill"):
        for n, ns in sorted(names.get(cat, {}).items(), key=lambda kv: -kv[1])[:6]:
            out.append(f"  {cat:10s} {ns / 1e6 / steps:8.2f}  {n}")
    return "\n".join(out)


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("csv", nargs="?", help="--stats kernel_stats.csv (whole run)")
    p.add_argument("--trace", help="kernel_trace.csv (per dispatch)")
    p.add_argument("--markers", help="marker_api_trace.csv (roctx ranges)")
    p.add_argument("--range", default="bench.timed")
    p.add_argument("--steps", type=int, required=True)
    a = p.parse_args(argv)
    if a.trace:
        if not a.markers:
            p.error("--trace needs --markers")
        lo, hi = window(a.markers, a.range)
        print(breakdown(from_trace(a.trace, lo, hi), a.steps, hi - lo))
    elif a.csv:
        print(breakdown(from_stats(a.csv), a.steps))
    else:
        p.error("give a --stats CSV or --trace + --markers")


if __name__ == "__main__":
    main()
