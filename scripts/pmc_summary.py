#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV output dirs per kernel (mean per dispatch +
derived ratios).  Thin wrapper over mxk8s.validate.profile.

    python scripts/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 [--filter gemm]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mxk8s.validate.profile import format_text, summarize  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("dirs", nargs="+")
ap.add_argument("--filter", default="")
a = ap.parse_args()
sys.stdout.write(format_text(summarize(a.dirs, a.filter)))
