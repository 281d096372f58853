#!/usr/bin/env bash
# PMC counters for the GEMM schedules (separate passes, --kernel-trace only).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$R${PYTHONPATH:+:$PYTHONPATH}
cd /tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P2="SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum"
SZ=${SIZES:-8192}
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P1 --output-format csv -d $R/gpurun_out/pmc1 -o run -- \
  python3 -m mxk8s.validate.gemm --sizes $SZ --variants ${VARIANTS:-all} --iters 12 --rounds 2 --warmup-s 0.5 > $R/gpurun_out/pmc1.log 2>&1
rc=$?; echo "pmc1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P2 --output-format csv -d $R/gpurun_out/pmc2 -o run -- \
  python3 -m mxk8s.validate.gemm --sizes $SZ --variants ${VARIANTS:-all} --iters 12 --rounds 2 --warmup-s 0.5 > $R/gpurun_out/pmc2.log 2>&1
rc=$?; echo "pmc2 rc=$rc"; exit $rc
