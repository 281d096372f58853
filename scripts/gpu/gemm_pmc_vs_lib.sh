#!/usr/bin/env bash
# PMC counters: hand-written GEMM (default schedule) vs hipBLASLt, 8192^3.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
mkdir -p gpurun_out
VARIANTS=5 SIZES=8192 bash scripts/gpu/gemm_pmc.sh || exit $?
python3 -m mxk8s.validate.profile --summarize gpurun_out/pmc1 gpurun_out/pmc2 > gpurun_out/pmc_vs_lib.txt
grep -E "^==|median|mfma_busy|clock|wait_any|wait_inst_any|active_inst|l2_hit|SQ_INSTS_LDS|SQ_WAIT_INST_LDS" gpurun_out/pmc_vs_lib.txt | grep -B1 -A9 "w4b\|Cijk" | head -40
