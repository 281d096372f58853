#!/usr/bin/env bash
# Both kernel libraries after moving the attention forward A/B variants
# (5-9) into the experiments build: the GPU tier on the production library
# (variants 5-9 skip), then the attention forward tests on the experiments
# library (every variant runs).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${1:-gpurun_out/r3libs}
mkdir -p "$OUT"
export PYTHONPATH=.
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu_prod.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_gpu_prod.log"; [ $rc -eq 0 ] || exit $rc
MXK_KERNELS_LIB=$PWD/mxk8s/_lib/libmxkernels_exp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_attention.py -k fwd -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_attn_exp.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_attn_exp.log"; exit $rc
