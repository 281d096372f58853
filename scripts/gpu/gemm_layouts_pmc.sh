#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
mkdir -p gpurun_out
export PYTHONPATH=$R${PYTHONPATH:+:$PYTHONPATH}
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/glpmc -o run -- python3 $R/scripts/gemm_layouts_bench.py > $R/gpurun_out/glpmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R && python3 -m mxk8s.validate.profile --summarize gpurun_out/glpmc --filter gemm_bf16_x > gpurun_out/glpmc_summary.txt
cat gpurun_out/glpmc_summary.txt
