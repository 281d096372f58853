#!/usr/bin/env bash
# Round 3: same-box A/B of the Llama-3-8B DDP step (current vs hipBLASLt
# forward vs unfused up-projection, interleaved), then a steady-state kernel
# trace of the current step bounded by the bench.timed roctx range.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
OUT=${1:-gpurun_out/r3_ddp}
mkdir -p "$OUT"
export PYTHONPATH=$R
run() {   # variant tag
  echo "== $1 ($2)" >> "$OUT/ab.log"
  timeout -k 10 300 python -u scripts/gpu/ddp_ab.py "$1" --steps 8 --warmup 3 > "$OUT/ab_$2.log" 2>&1 &&
    tail -1 "$OUT/ab_$2.log" >> "$OUT/ab.log"
}
run current 1 && run hipblaslt_fwd 2 && run unfused_w13 3 && run current 4 && run hipblaslt_fwd 5 &&
  run current 6 && (
  export TMPDIR=/tmp
  cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv \
    -d "$R/$OUT/prof" -o run -- python3 "$R/bench.py" --mode ddp --steps 4 --warmup 2 \
    > "$R/$OUT/prof.log" 2>&1)
