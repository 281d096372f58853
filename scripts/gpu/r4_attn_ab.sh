#!/bin/bash
# Attention A/B of two kernel libraries on one box: correctness of B, then
# the B=8 Llama-shape timings alternated A B A B.
#   scripts/gpu/r4_attn_ab.sh <libA> <libB> <outdir>
set -euo pipefail
A=$1; B=$2; OUT=$3
mkdir -p "$OUT"
MXK_KERNELS_LIB=$B timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_attention.py > "$OUT/pytest_B.log" 2>&1
for rep in 1 2; do
  for L in A B; do
    lib=$A; [ $L = B ] && lib=$B
    MXK_KERNELS_LIB=$lib BATCH=8 timeout -k 10 180 python -u scripts/attn_mxk_bench.py \
      | sed "s/^RESULT /RESULT $L$rep /" >> "$OUT/bench.log"
  done
done
