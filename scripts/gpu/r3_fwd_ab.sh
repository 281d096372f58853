#!/usr/bin/env bash
# Same-box DDP step A/B: every GEMM hand-written (default) vs the forward
# products on hipBLASLt (MXK_FWD_LIB=1 MXK_FUSED_W13=0, TunableOp table
# loaded), interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${1:-gpurun_out/r3fwdab}
mkdir -p "$OUT"
export PYTHONPATH=.
run() {   # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --mode ddp --steps 8 --warmup 3 > "$OUT/$tag.json" 2> "$OUT/$tag.err"
  local rc=$?
  echo "$tag rc=$rc $(python3 -c "import json,sys; d=json.loads(open('$OUT/$tag.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  return $rc
}
run mxk_1 MXK_NOP=1 && run lib_1 MXK_FWD_LIB=1 MXK_FUSED_W13=0 && \
run mxk_2 MXK_NOP=1 && run lib_2 MXK_FWD_LIB=1 MXK_FUSED_W13=0
