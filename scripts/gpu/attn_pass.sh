#!/bin/bash
# Attention GPU pass: the attention GPU tests (-k filter), the B = 8 timing
# (scripts/attn_mxk_bench.py) and, with PMC=1, three counter passes over
# attn_run.py (one rocprofv3 process each).  OUT=gpurun_out/<name>.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${OUT:-gpurun_out/r5_attn}
mkdir -p $OUT
export PYTHONPATH=$PWD TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_attention.py -k "${PYTEST_K:-v6 or variants or onepass or fwd_matches}" > $OUT/pytest.out 2>&1
rc=$?; echo pytest rc=$rc; tail -3 $OUT/pytest.out; [ $rc -eq 0 ] || exit $rc
BATCH=8 timeout -k 10 300 python3 -u scripts/attn_mxk_bench.py > $OUT/bench_b8.out 2>&1
rc=$?; echo bench rc=$rc; grep RESULT $OUT/bench_b8.out; [ $rc -eq 0 ] || exit $rc
if [ "${PMC:-0}" = 1 ]; then
  P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
  P2="SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum"
  P3="FETCH_SIZE GRBM_GUI_ACTIVE"
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    ( cd /tmp && BWD_VARIANTS=${BWD_VARIANTS:-5,6,7,8} timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P \
        --output-format csv -d $GRAFT_REPO_ROOT/$OUT/pmc$i -o run -- python3 $GRAFT_REPO_ROOT/scripts/gpu/attn_run.py ) \
      > $OUT/pmc_pass$i.log 2>&1
    rc=$?; echo pmc$i rc=$rc; [ $rc -eq 0 ] || exit $rc
  done
  python3 -c "
from mxk8s.validate.profile import summarize, format_text
import glob
print(format_text(summarize(sorted(glob.glob('$OUT/pmc*/')), 'attn')))" > $OUT/pmc_summary.txt 2>&1
  head -80 $OUT/pmc_summary.txt
fi
