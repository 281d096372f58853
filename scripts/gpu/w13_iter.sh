#!/usr/bin/env bash
# Persistent fused up-projection A/B (experiments library): numerics, then
# the kernel timing at the step shape.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=${1:-gpurun_out/w13}
mkdir -p "$O"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
export MXK_KERNELS_LIB=$PWD/mxk8s/_lib/libmxkernels_exp.so
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_mlp_fused.py -x -q -k "w13" --timeout 120 --timeout-method thread > "$O/test.log" 2>&1
rc=$?; echo "w13 tests rc=$rc: $(tail -1 "$O/test.log")"; [ $rc -eq 0 ] || { tail -30 "$O/test.log"; exit $rc; }
timeout -k 10 300 python3 -u scripts/gpu/w13_ab.py > "$O/ab.txt" 2>&1
rc=$?; echo "w13 ab rc=$rc"; grep RESULT "$O/ab.txt"; exit $rc
