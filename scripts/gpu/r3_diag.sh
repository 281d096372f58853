#!/usr/bin/env bash
# (1) attention forward timing ablations of the ping-pong kernel (7: no
#     softmax VALU, 8: no MFMAs) against 4 and 5;
# (2) L2-miss bytes (FETCH_SIZE) of the TN kernel vs hipBLASLt at K = 16384
#     for 1, 4 and 16 rounds of 256 tiles (does the per-tile miss volume
#     grow with the number of rounds?).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
OUT=$R/${1:-gpurun_out/r3diag}
mkdir -p "$OUT"
export PYTHONPATH=$R TMPDIR=/tmp
# forward variants 5-9 are A/B records: experiments library (make gemm-exp)
export MXK_KERNELS_LIB=${MXK_KERNELS_LIB:-$PWD/mxk8s/_lib/libmxkernels_exp.so}
VARIANTS=4,5,7,8 timeout -k 10 200 python3 -u scripts/gpu/attn_fwd_ab.py > $OUT/attn_diag.log 2>&1 || exit $?
grep RESULT $OUT/attn_diag.log
cd /tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/fetch -o run -- python3 -m mxk8s.validate.gemm --sizes 16384 --shapes 4096x4096x16384,8192x8192x16384 --iters 6 --rounds 2 --warmup-s 0.5 > $OUT/fetch.log 2>&1
rc=$?
echo "fetch rc=$rc"
exit $rc
