#!/usr/bin/env bash
# Cycle stamps of forward variant 10 from alternative kernel libraries
# (MXK_KERNELS_LIB), default library first.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=${1:-gpurun_out/fwd10_libab}
shift
mkdir -p "$O"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
timeout -k 10 180 python3 -u scripts/gpu/fwd10_stamps.py > "$O/stamps_default.txt" 2>&1
rc=$?; echo "default rc=$rc"; grep "per tile\|median per wave" "$O/stamps_default.txt"; [ $rc -eq 0 ] || exit $rc
for L in "$@"; do
  n=$(basename "$L" .so)
  MXK_KERNELS_LIB=$PWD/$L timeout -k 10 180 python3 -u scripts/gpu/fwd10_stamps.py > "$O/stamps_$n.txt" 2>&1
  rc=$?; echo "$n rc=$rc"; grep "per tile\|median per wave" "$O/stamps_$n.txt"; [ $rc -eq 0 ] || exit $rc
  MXK_KERNELS_LIB=$PWD/$L timeout -k 10 120 python3 -u -m pytest tests/test_gpu_attention.py -q -x -k "fwd and 10" --timeout 60 > "$O/test_$n.txt" 2>&1
  rc=$?; echo "$n fwd tests rc=$rc: $(tail -1 "$O/test_$n.txt")"
done
