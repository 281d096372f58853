#!/usr/bin/env bash
# Operand-swizzle A/B of the default GEMM schedule: 26 (full XOR swizzle on
# the DMA source, conflict-free reads) vs 37 (linear) vs 38 (64-B halves
# only): correctness, timing at the protocol sizes, then one PMC pass
# (waits, LDS bank conflicts, MFMA busy) at 8192^3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
OUT=$R/${1:-gpurun_out/r3swz}
mkdir -p "$OUT"
export PYTHONPATH=$R MXK_KERNELS_LIB=$R/mxk8s/_lib/libmxkernels_exp.so TMPDIR=/tmp
timeout -k 10 200 python3 -u scripts/gpu/ring_check.py 26,38,39,40 > "$OUT/check.log" 2>&1 && \
timeout -k 10 500 python3 -u -m mxk8s.validate.gemm --sizes 8192,4096,16384 --variants 26,38,39,40 --iters 96 --rounds 16 > "$OUT/gemm_ab.log" 2>&1 && \
( cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc -o run -- python3 -m mxk8s.validate.gemm --sizes 8192 --variants 26,38,39,40 --iters 12 --rounds 2 --warmup-s 0.5 > $OUT/pmc.log 2>&1 )
rc=$?
tail -1 "$OUT/check.log"
grep RESULT "$OUT/gemm_ab.log" | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l.split('RESULT ', 1)[1]); print(d['kernel'], d['M'], round(d['tflops_median'], 1))"
exit $rc
