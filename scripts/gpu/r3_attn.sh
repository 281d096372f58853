#!/usr/bin/env bash
# Attention forward ping-pong variants 5 / 6 (6 = MFMA phase at raised
# priority): GPU numerics of every forward variant, then the Llama-3-8B-shape
# A/B (causal and full) against variant 4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${1:-gpurun_out/r3a}
mkdir -p "$OUT"
export PYTHONPATH=.
# forward variants 5-9 are A/B records: experiments library (make gemm-exp)
export MXK_KERNELS_LIB=${MXK_KERNELS_LIB:-$PWD/mxk8s/_lib/libmxkernels_exp.so}
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -k fwd -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_fwd.log" 2>&1 && \
VARIANTS=4,5,6 timeout -k 10 200 python -u scripts/gpu/attn_fwd_ab.py > "$OUT/fwd_ab.log" 2>&1 && \
CAUSAL=0 VARIANTS=4,5,6 timeout -k 10 200 python -u scripts/gpu/attn_fwd_ab.py > "$OUT/fwd_ab_full.log" 2>&1
rc=$?
tail -3 "$OUT/pytest_fwd.log"; grep RESULT "$OUT"/fwd_ab*.log
exit $rc
