#!/usr/bin/env bash
# Attention backward (variant 9) from the default kernel library against an
# alternative one (MXK_KERNELS_LIB): outputs bit for bit, then alternating
# timing runs (separate processes, same box), then dK / dV cycle stamps.
#   bash scripts/gpu/bwd_lib_ab.sh OUT_DIR mxk8s/_lib/libmxkernels_X.so
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=${1:-gpurun_out/bwd_lib_ab}
ALT=$2
mkdir -p "$O"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_attention.py -x -q -k "bwd" --timeout 120 --timeout-method thread > "$O/test.log" 2>&1
rc=$?; echo "bwd tests rc=$rc: $(tail -1 "$O/test.log")"; [ $rc -eq 0 ] || exit $rc
rm -f "$O/ref.pt"
for r in 1 2 3; do
  MXK_KERNELS_LIB=$PWD/$ALT SAVE=$O/ref.pt VARIANTS=9 timeout -k 10 120 python3 -u scripts/gpu/attn_bwd_ab.py > "$O/alt_$r.txt" 2>&1
  rc=$?; echo "alt $r rc=$rc: $(grep RESULT "$O/alt_$r.txt" | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
  SAVE=$O/ref.pt VARIANTS=9 timeout -k 10 120 python3 -u scripts/gpu/attn_bwd_ab.py > "$O/new_$r.txt" 2>&1
  rc=$?; echo "new $r rc=$rc: $(grep RESULT "$O/new_$r.txt" | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 180 python3 -u scripts/gpu/bwd256_stamps.py > "$O/stamps.txt" 2>&1
rc=$?; echo "stamps rc=$rc"; cat "$O/stamps.txt"; exit $rc
