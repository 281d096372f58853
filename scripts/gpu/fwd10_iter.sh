#!/usr/bin/env bash
# Forward variant 10 iteration: numerics (forward tests), cycle stamps, and
# the 4 vs 10 A/B at the step shape (causal and full).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=${1:-gpurun_out/fwd10}
mkdir -p "$O"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_attention.py -x -q -k "fwd" --timeout 120 --timeout-method thread > "$O/test.log" 2>&1
rc=$?; echo "fwd tests rc=$rc"; tail -5 "$O/test.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python3 -u scripts/gpu/fwd10_stamps.py > "$O/stamps.txt" 2>&1
rc=$?; echo "stamps rc=$rc"; cat "$O/stamps.txt"; [ $rc -eq 0 ] || exit $rc
VARIANTS=4,10 timeout -k 10 180 python3 -u scripts/gpu/attn_fwd_ab.py > "$O/ab_causal.txt" 2>&1
rc=$?; echo "ab causal rc=$rc"; grep RESULT "$O/ab_causal.txt"; [ $rc -eq 0 ] || exit $rc
CAUSAL=0 VARIANTS=4,10 timeout -k 10 180 python3 -u scripts/gpu/attn_fwd_ab.py > "$O/ab_full.txt" 2>&1
rc=$?; echo "ab full rc=$rc"; grep RESULT "$O/ab_full.txt"; exit $rc
