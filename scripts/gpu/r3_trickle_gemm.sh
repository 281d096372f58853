#!/usr/bin/env bash
# Trickle-store GEMMs: correctness (schedules 26/31/32, the x2t GPU tests),
# then A/B timing (TN schedules vs the no-store ablation 10 and hipBLASLt;
# layout kernel variant 1 vs x2t on the Llama-3-8B step shapes).  Each GPU
# step has its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${1:-gpurun_out/r3g}
mkdir -p "$OUT"
export PYTHONPATH=.
EXP=mxk8s/_lib/libmxkernels_exp.so
export MXK_KERNELS_LIB=$EXP   # the trickle-store kernels are experiments-only
timeout -k 10 200 python -u scripts/gpu/ring_check.py 26,31 > "$OUT/check.log" 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "trickle or every_schedule or headline" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_trickle.log" 2>&1 && \
timeout -k 10 400 python -u -m mxk8s.validate.gemm --sizes 8192,4096,16384 --variants 26,31 --iters 96 --rounds 12 > "$OUT/gemm_ab.log" 2>&1 && \
TOKENS=16384 VARIANTS=1,4 timeout -k 10 400 python -u scripts/gemm_layouts_bench.py > "$OUT/layouts_ab.log" 2>&1
