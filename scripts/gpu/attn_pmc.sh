#!/bin/bash
# Counter passes over attn_run.py only (FWD_VARIANTS / BWD_VARIANTS select
# the kernels): three rocprofv3 --pmc runs, one process each, then the
# per-kernel summary.  OUT=gpurun_out/<name>.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${OUT:-gpurun_out/r5_pmc}
mkdir -p $OUT
export PYTHONPATH=$PWD TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P2="SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_ACTIVE_INST_VALU TCC_HIT_sum TCC_MISS_sum"
P3="FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  ( cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P \
      --output-format csv -d $GRAFT_REPO_ROOT/$OUT/pmc$i -o run -- python3 $GRAFT_REPO_ROOT/scripts/gpu/attn_run.py ) \
    > $OUT/pmc_pass$i.log 2>&1
  rc=$?; echo pmc$i rc=$rc; [ $rc -eq 0 ] || exit $rc
done
python3 -c "
from mxk8s.validate.profile import summarize, format_text
import glob
print(format_text(summarize(sorted(glob.glob('$OUT/pmc*/')), 'attn')))" > $OUT/pmc_summary.txt 2>&1
cat $OUT/pmc_summary.txt
