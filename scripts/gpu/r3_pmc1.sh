#!/usr/bin/env bash
# PMC passes (--kernel-trace only, one process each): attention forward
# variant 4 vs 5 (VALU/MFMA co-execution, waits, LDS), the non-causal
# forward A/B, and the GEMM at 8192^3 / 16384^3 (default schedule vs
# hipBLASLt: HBM fetch bytes, L2 hits, MFMA busy).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
OUT=$R/${1:-gpurun_out/r3pmc}
mkdir -p "$OUT"
export PYTHONPATH=$R TMPDIR=/tmp
# forward variants 5-9 are A/B records: experiments library (make gemm-exp)
export MXK_KERNELS_LIB=${MXK_KERNELS_LIB:-$PWD/mxk8s/_lib/libmxkernels_exp.so}
step() {
  local name=$1 secs=$2
  shift 2
  ( cd /tmp && timeout -s KILL "$secs" "$@" ) > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "$OUT/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
AV="SQ_VALU_MFMA_COEXEC_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
AW="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
G1="SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
G2="FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE"
step attn_av 90 env FWD_VARIANTS=4,5 ITERS=3 rocprofv3 --kernel-trace --pmc $AV --output-format csv -d $OUT/attn_av -o run -- python3 $R/scripts/gpu/attn_run.py
step attn_aw 90 env FWD_VARIANTS=4,5 ITERS=3 rocprofv3 --kernel-trace --pmc $AW --output-format csv -d $OUT/attn_aw -o run -- python3 $R/scripts/gpu/attn_run.py
step attn_ab_noncausal 200 env CAUSAL=0 VARIANTS=4,5 python3 -u $R/scripts/gpu/attn_fwd_ab.py
step gemm_g1 120 rocprofv3 --kernel-trace --pmc $G1 --output-format csv -d $OUT/gemm_g1 -o run -- python3 -m mxk8s.validate.gemm --sizes 8192,16384 --iters 12 --rounds 2 --warmup-s 0.5
step gemm_g2 120 rocprofv3 --kernel-trace --pmc $G2 --output-format csv -d $OUT/gemm_g2 -o run -- python3 -m mxk8s.validate.gemm --sizes 8192,16384 --iters 12 --rounds 2 --warmup-s 0.5
python3 -m mxk8s.validate.profile --summarize $OUT/attn_av $OUT/attn_aw > $OUT/attn_summary.txt 2>&1
python3 -m mxk8s.validate.profile --summarize $OUT/gemm_g1 $OUT/gemm_g2 > $OUT/gemm_summary.txt 2>&1
echo done
