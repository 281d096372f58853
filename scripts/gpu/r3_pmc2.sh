#!/usr/bin/env bash
# L2-miss bytes (FETCH_SIZE) and cycles of the TN schedules at 16384^3:
# default 26 (one workgroup per tile) vs the persistent ones (11, 12, 31)
# vs hipBLASLt's stream-K kernel; --kernel-trace only, one pass each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
OUT=$R/${1:-gpurun_out/r3pmc2}
mkdir -p "$OUT"
export PYTHONPATH=$R TMPDIR=/tmp MXK_KERNELS_LIB=$R/mxk8s/_lib/libmxkernels_exp.so
G2="FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE"
G1="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
cd /tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $G2 --output-format csv -d $OUT/g2 -o run -- python3 -m mxk8s.validate.gemm --sizes 16384 --variants 26,11,12,31 --iters 6 --rounds 2 --warmup-s 0.5 > $OUT/g2.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $G1 --output-format csv -d $OUT/g1 -o run -- python3 -m mxk8s.validate.gemm --sizes 16384 --variants 26,11,12,31 --iters 6 --rounds 2 --warmup-s 0.5 > $OUT/g1.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
