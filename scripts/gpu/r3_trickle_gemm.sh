#!/usr/bin/env bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${1:-gpurun_out/r3g}
mkdir -p "$OUT"
export PYTHONPATH=.
EXP=mxk8s/_lib/libmxkernels_exp.so
MXK_KERNELS_LIB=$EXP timeout -k 10 200 python -u scripts/gpu/ring_check.py 26,31,32 > "$OUT/check.log" 2>&1 && \
MXK_KERNELS_LIB=$EXP timeout -k 10 400 python -u -m mxk8s.validate.gemm --sizes 8192,4096,16384 --variants 26,31,32,10 --iters 96 --rounds 12 > "$OUT/gemm_ab.log" 2>&1
[ $? -eq 0 ] && TOKENS=16384 VARIANTS=1,4 timeout -k 10 400 python -u scripts/gemm_layouts_bench.py > "$OUT/layouts_ab.log" 2>&1
