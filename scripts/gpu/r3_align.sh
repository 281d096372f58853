#!/usr/bin/env bash
# Code-placement A/B of the default GEMM schedule: 26 (K-loop head at 48 mod
# 64 B) vs 33-36 (16 / 0 / 28 / 4 mod 64), correctness sweep first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${1:-gpurun_out/r3al}
mkdir -p "$OUT"
export PYTHONPATH=. MXK_KERNELS_LIB=mxk8s/_lib/libmxkernels_exp.so
timeout -k 10 200 python -u scripts/gpu/ring_check.py 26,33,34,35,36 > "$OUT/check.log" 2>&1 && \
timeout -k 10 500 python -u -m mxk8s.validate.gemm --sizes 8192,4096,16384 --variants 26,33,34,35,36 --iters 96 --rounds 12 > "$OUT/gemm_ab.log" 2>&1
rc=$?
tail -1 "$OUT/check.log"
grep RESULT "$OUT/gemm_ab.log" | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l.split('RESULT ', 1)[1]); print(d['kernel'], d['M'], round(d['tflops_median'], 1))"
exit $rc
