#!/usr/bin/env bash
# Attention bench + per-kernel stats + PMC counters of the attention kernels.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
mkdir -p gpurun_out
export PYTHONPATH=$R${PYTHONPATH:+:$PYTHONPATH}
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/attn_mxk_bench.py > gpurun_out/attn_bench.log 2>&1
rc=$?; echo "attn bench rc=$rc"; grep RESULT gpurun_out/attn_bench.log; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/attn_ks -o run -- python3 $R/scripts/attn_mxk_bench.py > $R/gpurun_out/attn_ks.log 2>&1
rc=$?; echo "ks rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU --output-format csv -d $R/gpurun_out/attn_pmc -o run -- python3 $R/scripts/attn_mxk_bench.py > $R/gpurun_out/attn_pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R && python3 -m mxk8s.validate.profile --summarize gpurun_out/attn_pmc --filter attn > gpurun_out/attn_pmc_summary.txt
cat gpurun_out/attn_pmc_summary.txt | grep -E "==|median|mfma|lds_bank|clock|wait_any"
find gpurun_out/attn_ks -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/attn_kernel_stats.csv
