#!/usr/bin/env bash
# Attention forward variant 5 (8-wave ping-pong): GPU numerics of every
# forward variant, then the Llama-3-8B-shape A/B (4 vs 5, bit-identity).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${1:-gpurun_out/r3a}
mkdir -p "$OUT"
export PYTHONPATH=.
timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -k fwd -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_fwd.log" 2>&1 && \
VARIANTS=4,5 timeout -k 10 200 python -u scripts/gpu/attn_fwd_ab.py > "$OUT/fwd_ab.log" 2>&1
