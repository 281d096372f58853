#!/bin/bash
# Counter passes (one process each, --kernel-trace only) over attn_run.py.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/attn_pmc
mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P2="SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum"
P3="FETCH_SIZE GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/pmc$i -o run -- python3 scripts/gpu/attn_run.py > $OUT/pass$i.log 2>&1
done
python3 -c "
from mxk8s.validate.profile import summarize, format_text
import glob
print(format_text(summarize(sorted(glob.glob('$OUT/pmc*')), 'attn')))" > $OUT/summary.txt
