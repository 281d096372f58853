# Same-box A/B of the Llama-3-8B step (bench.py --mode ddp): TN default 52 vs
# the round-3 default 26 (MXK_TN_VARIANT) and the w13 SwiGLU kernel on the
# one-barrier loop (MXK_W13_SCHED=1) and the dgrad-SwiGLU epilogue without its
# g/u prefetch (MXK_SWIGLU_WIDE=5), interleaved twice.  Second set: layout
# kernel B-outer order (MXK_X2_ORDER=1), w13 non-temporal gu stores
# (MXK_W13_SCHED=2), attention backward variant 3 (MXK_ATTN_BWD_VARIANT=3).
# Set 3: the dgrad-SwiGLU GEMM staggered by XCD group (MXK_SWIGLU_WIDE=8).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r4step; mkdir -p $O
export PYTHONPATH=.
# the A/B switches below are built into the experiments library only
export MXK_KERNELS_LIB=$PWD/mxk8s/_lib/libmxkernels_exp.so
run() {  # name env...
  local n=$1; shift
  timeout -k 10 240 env "$@" python3 bench.py --mode ddp --steps 8 --warmup 3 > $O/$n.out 2> $O/$n.err || return $?
  python3 -c "
import json,sys
for l in open('$O/$n.out'):
    if l.startswith('{'):
        d=json.loads(l); print('$n', d['value'], d['ms_per_step'])"
}
for r in 1 2; do
  run base$r MXK_NOP=1 && run swstag_$r MXK_SWIGLU_WIDE=8 || exit $?
done
