#!/bin/bash
# TN schedules at the step's forward shapes vs hipBLASLt (validator A/B)
set -euo pipefail
OUT=${1:-gpurun_out/r4fwdshapes}
mkdir -p "$OUT"
MXK_KERNELS_LIB=$PWD/mxk8s/_lib/libmxkernels_exp.so timeout -k 10 600 python -u -m mxk8s.validate.gemm \
  --sizes "" --shapes 16384x4096x4096,16384x6144x4096,16384x4096x14336,16384x28672x4096 \
  --variants 52,26,47,6,9,1,27,28 --rounds 4 --iters 40 > "$OUT/fwd_shapes.log" 2>&1
