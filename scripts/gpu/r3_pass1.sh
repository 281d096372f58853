#!/usr/bin/env bash
# Round-3 first pass after the session restart: trickle-store schedules'
# correctness sweep, TN schedule A/B (26 vs trickle 31/32 vs hipBLASLt),
# layout-kernel A/B (variant 1 vs x2t 4) on the Llama-3-8B step shapes, the
# headline bench, the DDP step, the full GPU test tier (incl. the ping-pong
# attention forward, variant 5) and the attention forward A/B (4 vs 5).
# Each GPU step has its own time limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${1:-gpurun_out/r3p1}
mkdir -p "$OUT"
export PYTHONPATH=.
EXP=mxk8s/_lib/libmxkernels_exp.so
step() {   # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -3 "$OUT/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
step ring_check 200 env MXK_KERNELS_LIB=$EXP python -u scripts/gpu/ring_check.py 26,31,32
step gemm_ab 400 env MXK_KERNELS_LIB=$EXP python -u -m mxk8s.validate.gemm --sizes 8192,4096,16384 --variants 26,31,32 --iters 96 --rounds 12
step layouts_ab 400 env TOKENS=16384 VARIANTS=1,4 python -u scripts/gemm_layouts_bench.py
step bench 300 python -u bench.py --steps 20 --warmup 5
step bench_ddp 400 python -u bench.py --mode ddp --steps 10 --warmup 3
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step attn_fwd_ab 200 env VARIANTS=4,5 python -u scripts/gpu/attn_fwd_ab.py
