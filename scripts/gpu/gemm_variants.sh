#!/usr/bin/env bash
# A/B the GEMM schedules in one process on random data.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -m mxk8s.validate.gemm --sizes ${SIZES:-8192,4096} --variants all \
    --iters 60 --rounds 6 > gpurun_out/gemm_variants.log 2>&1
rc=$?; echo "gemm rc=$rc"; grep RESULT gpurun_out/gemm_variants.log | python3 -c "
import sys, json
for l in sys.stdin:
    r = json.loads(l[7:]); print(f\"{r['kernel']:14s} {r['M']:6d} {r['tflops_median']:8.1f} TF (best {r['tflops_best']:.1f})\")
"; exit $rc
