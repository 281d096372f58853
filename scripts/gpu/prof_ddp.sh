#!/usr/bin/env bash
# Steady-state kernel profile of the Llama-3-8B DDP step (world size 1):
# kernel trace + roctx markers, then the per-category breakdown of the
# dispatches inside the bench.timed range.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
O=${1:-gpurun_out/prof_ddp}
STEPS=${STEPS:-4}
mkdir -p "$R/$O"
export TMPDIR=/tmp
export PYTHONPATH=$R${PYTHONPATH:+:$PYTHONPATH}
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv \
  -d "$R/$O/trace" -o run -- python3 "$R/bench.py" --mode ddp --steps "$STEPS" --warmup 2 \
  > "$R/$O/prof.out" 2> "$R/$O/prof.err"
rc=$?; echo "prof rc=$rc"; tail -1 "$R/$O/prof.out"
[ $rc -eq 0 ] || exit $rc
cd "$R"
KT=$(find "$O/trace" -name '*kernel_trace.csv' | head -1)
MT=$(find "$O/trace" -name '*marker_api_trace.csv' | head -1)
python3 scripts/kernel_breakdown.py --trace "$KT" --markers "$MT" --range bench.timed --steps "$STEPS" \
  > "$O/breakdown.txt" 2>&1
rc=$?; cat "$O/breakdown.txt" | head -30; exit $rc
