#!/bin/bash
# Step GEMM products isolated vs hipBLASLt (scripts/step_gemm_vs_hipblaslt.py)
set -euo pipefail
OUT=${1:-gpurun_out/r4shapes}
mkdir -p "$OUT"
timeout -k 10 600 python -u scripts/step_gemm_vs_hipblaslt.py > "$OUT/step_shapes.log" 2>&1
