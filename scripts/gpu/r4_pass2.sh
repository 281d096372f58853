#!/usr/bin/env bash
# Round-4 GPU pass: GPU tier on the pruned production library, GEMM A/B of
# the production kernel's own template (26) vs the experiments template (46)
# and the K-rotated tile order (44), stamps, the headline bench, the
# contention rehearsal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=${1:-gpurun_out/r4p2}
mkdir -p $O
bash scripts/gpu/pass.sh $O pytest bench || exit $?
VARIANTS=26,46,44,6 bash scripts/gpu/probe_map.sh $O/map || exit $?
MXK_KERNELS_LIB=$PWD/mxk8s/_lib/libmxkernels_exp.so PYTHONPATH=. timeout -k 10 300 python3 -u scripts/gpu/gemm_stamps.py > $O/stamps.log 2>&1 || exit $?
cat $O/stamps.log
CONT_CUS=16,32,64 bash scripts/gpu/pass.sh $O contention
