#!/usr/bin/env bash
# End-of-round pass (round 3): the GPU test tier, smoke(), the headline bench
# at the driver's arguments, the DDP step, then the DDP step's steady-state
# kernel breakdown (kernel trace bounded by the bench.timed roctx range).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=${1:-gpurun_out/r3final}
bash scripts/gpu/final_check.sh "$O" || exit $?
STEPS=3 bash scripts/gpu/prof_ddp.sh "$O/prof_ddp" || exit $?
KT=$(find "$O/prof_ddp/trace" -name '*kernel_trace.csv' | head -1)
echo "library GEMM dispatches in the trace: $(grep -c 'Cijk' "$KT" || true)"
