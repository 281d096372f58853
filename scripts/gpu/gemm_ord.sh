#!/usr/bin/env bash
# Schedule A/B of the w4b GEMM: default (6) vs exact-LDS-wait variants (13, 15),
# bitwise output check against the default, then the s_memtime stamps of 12/14.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 120 python3 - <<'PY' || exit 1
import torch
from mxk8s.ops import _lib
L = _lib.lib(); dev = torch.device("cuda")
import os; VARS = [int(x) for x in os.environ.get("CHECK", "6,13,15").split(",")]
for n in (4096, 8192):
    A = (torch.rand(n, n, device=dev) * 2 - 1).bfloat16(); B = (torch.rand(n, n, device=dev) * 2 - 1).bfloat16()
    outs = {}
    for v in VARS:
        C = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
        _lib.check(L.mxk_gemm_bf16_tn_variant(A.data_ptr(), B.data_ptr(), C.data_ptr(), n, n, n, n, n, n, v, _lib.stream_ptr(dev)), "v")
        outs[v] = C
    torch.cuda.synchronize()
    ref = (A.float() @ B.float().t())
    for v, C in outs.items():
        print(f"n={n} v{v} bitwise_eq_v6={torch.equal(C, outs[6])} max_rel={((C.float()-ref).abs().max()/ref.abs().max()).item():.2e}")
PY
timeout -k 10 400 python3 -m mxk8s.validate.gemm --sizes ${SIZES:-8192,4096} --variants ${VARIANTS:-6,13,15} \
    --iters 60 --rounds 8 > gpurun_out/gemm_ord.log 2>&1 || { echo "variants failed"; exit 1; }
grep RESULT gpurun_out/gemm_ord.log | python3 -c "
import sys, json
for l in sys.stdin:
    r = json.loads(l[7:]); print(f\"{r['kernel']:14s} {r['M']:6d} {r['tflops_median']:8.1f} TF (best {r['tflops_best']:.1f})\")
"
for v in ${STAMPS-12 14}; do
  STAMP_VARIANT=$v timeout -k 10 120 python3 scripts/gemm_stamps.py > gpurun_out/gemm_stamps_v$v.log 2>&1 || { echo "stamps $v failed"; exit 1; }
  grep RESULT gpurun_out/gemm_stamps_v$v.log
done
