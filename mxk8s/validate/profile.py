"""rocprofv3 counter pass for the GEMM validator (SURVEY.md §5 tracing row).

Counters perturb timing, so they are collected in SEPARATE processes, one
counter group per pass, each with `--kernel-trace` only (never combined with
sys/runtime traces):

    python -m mxk8s.validate --tests gemm --profile      (validator Job)
    python -m mxk8s.validate.profile --sizes 8192 --out DIR

ROCm 7.2 ships no gfx950 derived-counter XML, so the ratios below are
computed here from raw SQ/GRBM/TCC counters (MI355X_MICROARCH.md §PMC):

  MFMA busy / SIMD   SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 4 SIMDs * CUs)
  effective clock    GRBM_GUI_ACTIVE / 8 / kernel time  (8 XCDs summed)
  LDS conflicts      SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  L2 hit rate        TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

PASSES = (
    ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
     "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "GRBM_GUI_ACTIVE"),
    ("SQ_WAIT_INST_LDS", "SQ_LDS_UNALIGNED_STALL", "SQ_INSTS_LDS", "SQ_INSTS_MFMA",
     "TCC_HIT_sum", "TCC_MISS_sum"),
    # memory-side reads (MALL + HBM); gfx950 reports half the bytes of wide
    # streaming reads (MI355X_MICROARCH.md §HBM): compare ratios, not bytes
    ("FETCH_SIZE", "GRBM_GUI_ACTIVE"),
)
SIMDS = 256 * 4   # MI355X: 256 CUs x 4 SIMDs


def load(dirs, filt: str = ""):
    """Mean counter value per dispatch and kernel times from rocprofv3 CSVs."""
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = row.get("Kernel_Name", "")
                    if filt and filt not in k:
                        continue
                    per[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
        for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = row.get("Kernel_Name", "")
                    if filt and filt not in k:
                        continue
                    dur[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    return per, dur


def derive(m: dict, times: list) -> dict:
    """Utilisation ratios from mean raw counters + the kernel's dispatch times."""
    out = {}
    t = sorted(times)[len(times) // 2] if times else None
    if t:
        out["median_us"] = t * 1e6
    w = m.get("SQ_WAVE_CYCLES")
    if w:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in m:
                out[c.lower() + "_frac"] = m[c] / w
    g = m.get("GRBM_GUI_ACTIVE")
    if g and t:
        out["effective_clock_ghz"] = g / 8 / t / 1e9
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and g:
        out["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * SIMDS)
    if m.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_bank_conflict_frac"] = m.get("SQ_LDS_BANK_CONFLICT", 0.0) / m["SQ_LDS_IDX_ACTIVE"]
    if "TCC_HIT_sum" in m and "TCC_MISS_sum" in m and (m["TCC_HIT_sum"] + m["TCC_MISS_sum"]):
        out["l2_hit_rate"] = m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
    return out


def summarize(dirs, filt: str = "") -> dict:
    per, dur = load(dirs, filt)
    res = {}
    for k, cs in per.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        res[k] = {"counters": m, "derived": derive(m, dur.get(k, [])),
                  "dispatches": len(dur.get(k, []))}
    return res


def format_text(summary: dict) -> str:
    lines = []
    for k, s in summary.items():
        lines.append(f"== {k[:110]}")
        d = s["derived"]
        if "median_us" in d:
            lines.append(f"   dispatch time median {d['median_us']:.1f} us over {s['dispatches']} dispatches")
        for c in sorted(s["counters"]):
            lines.append(f"   {c:32s} {s['counters'][c]:.4g}")
        for c in sorted(d):
            if c != "median_us":
                lines.append(f"   {c:32s} {d[c]:.3f}")
    return "\n".join(lines) + "\n"


def profile_gemm(sizes: str, out_dir: str, variants: str = "", timeout: int = 240,
                 filt: str = "") -> dict:
    """Run the GEMM validator under rocprofv3 once per counter group."""
    rocprof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    dirs = []
    for i, counters in enumerate(PASSES):
        d = os.path.join(out_dir, f"pmc{i + 1}")
        # the program directly after `--` (no env/bash hop: the profiler's
        # preload has already initialised the GPU)
        cmd = [rocprof, "--kernel-trace", "--pmc", *counters, "--output-format", "csv",
               "-d", d, "-o", "run", "--", sys.executable, "-m", "mxk8s.validate.gemm",
               "--sizes", sizes, "--iters", "12", "--rounds", "2", "--warmup-s", "0.5"]
        if variants:
            cmd += ["--variants", variants]
        repo = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        pp = os.environ.get("PYTHONPATH", "")
        env = {**os.environ, "TMPDIR": os.environ.get("TMPDIR", "/tmp"),
               "PYTHONPATH": repo + (os.pathsep + pp if pp else "")}
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
        if p.returncode != 0:
            raise RuntimeError(f"rocprofv3 pass {i + 1} failed rc={p.returncode}: {p.stderr[-2000:]}")
        dirs.append(d)
    return summarize(dirs, filt)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--sizes", default="8192")
    ap.add_argument("--variants", default="")
    ap.add_argument("--out", default="gpurun_out/gemm_pmc")
    ap.add_argument("--summarize", nargs="*", help="only summarise existing rocprofv3 output dirs")
    ap.add_argument("--filter", default="")
    a = ap.parse_args(argv)
    if a.summarize:
        sys.stdout.write(format_text(summarize(a.summarize, a.filter)))
        return 0
    s = profile_gemm(a.sizes, a.out, a.variants, filt=a.filter)
    sys.stdout.write(format_text(s))
    for k, v in s.items():
        print("RESULT " + json.dumps({"test": "gemm_profile", "kernel": k[:120], **v["derived"]}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
