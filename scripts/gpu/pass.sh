#!/usr/bin/env bash
# One parameterised GPU pass (replaces the per-experiment one-off scripts).
#
#   bash scripts/gpu/pass.sh OUT STEP [STEP ...]
#
# Every step runs under its own time limit and writes OUT/<step>.out/.err;
# the first failing step ends the call (no GPU work after a fault/timeout).
# Steps (environment knobs in brackets):
#   pytest        the full GPU tier                       [PYTEST_K: -k filter]
#   pytest_exp    A/B-record kernels on the experiments library [PYTEST_K]
#   smoke         __graft_entry__.smoke()
#   bench         bench.py at the driver's arguments (--steps 20 --warmup 5)
#   bench_ddp     bench.py --mode ddp                      [DDP_STEPS, DDP_ENV]
#   gemm_ab       A/B of TN schedules                      [VARIANTS, SIZES, EXP=1]
#   layouts_ab    step-shape A/B of the layout kernel      [VARIANTS]
#   attn_ab       attention fwd/bwd timing                 [ATTN_ARGS]
#   prof_ddp      kernel trace + roctx breakdown of the DDP step [STEPS]
#   pmc_gemm      PMC counters of the TN GEMM              [VARIANTS, SIZES, COUNTERS]
#   contention    DDP step beside a CU-pinned HBM streamer  [CONT_CUS, CONT_PLACE]
#   ddp_gloo2     the multi-rank DDP step (ZeRO-1) rehearsed: 2 gloo ranks on one GPU,
#                 2 Llama-3-8B layers (NOT the headline config)
#   validator_gloo2  bench.py validator mode, 2 gloo ranks on one GPU
#   ddp_l2        the same 2-layer step on one rank (the reference for ddp_gloo2)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
O=$R/${1:?usage: pass.sh OUT STEP...}
shift
mkdir -p "$O"
export PYTHONPATH=$R${PYTHONPATH:+:$PYTHONPATH}
export TMPDIR=/tmp
EXP_LIB=$R/mxk8s/_lib/libmxkernels_exp.so
PYT="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider"

run() {   # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.out" 2> "$O/$name.err"
  local rc=$?
  echo "$name rc=$rc"
  tail -2 "$O/$name.out"
  [ $rc -eq 0 ] || exit $rc
}
prof() {  # name, seconds, rocprofv3 args... (run from /tmp; the program follows --)
  local name=$1 secs=$2
  shift 2
  ( cd /tmp && timeout -s KILL "$secs" rocprofv3 "$@" ) > "$O/$name.out" 2> "$O/$name.err"
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -eq 0 ] || exit $rc
}

for step in "$@"; do
  case $step in
    pytest)
      run pytest 900 $PYT tests -m gpu ${PYTEST_K:+-k "$PYTEST_K"} ;;
    pytest_exp)
      run pytest_exp 600 env MXK_KERNELS_LIB=$EXP_LIB $PYT tests -m gpu \
        -k "${PYTEST_K:-attn_fwd or schedule or trickle}" ;;
    smoke)
      run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)
      run bench 300 python3 bench.py --steps 20 --warmup 5 ;;
    bench_ddp)
      run bench_ddp 420 env ${DDP_ENV:-MXK_NOP=1} python3 bench.py --mode ddp \
        --steps "${DDP_STEPS:-10}" --warmup 3 ;;
    gemm_ab)
      run gemm_ab 500 env ${EXP:+MXK_KERNELS_LIB=$EXP_LIB} python3 -u -m mxk8s.validate.gemm \
        --sizes "${SIZES:-8192,4096,16384}" --variants "${VARIANTS:-26}" --iters 96 --rounds 12 ;;
    layouts_ab)
      run layouts_ab 400 env TOKENS=16384 VARIANTS="${VARIANTS:-1,4}" python3 -u scripts/gemm_layouts_bench.py ;;
    attn_ab)
      run attn_ab 300 python3 -u scripts/attn_mxk_bench.py ${ATTN_ARGS:-} ;;
    prof_ddp)
      prof prof_ddp 600 --kernel-trace --marker-trace --stats --output-format csv \
        -d "$O/prof_ddp" -o run -- python3 "$R/bench.py" --mode ddp --steps "${STEPS:-4}" --warmup 2
      KT=$(find "$O/prof_ddp" -name '*kernel_trace.csv' | head -1)
      MT=$(find "$O/prof_ddp" -name '*marker_api_trace.csv' | head -1)
      python3 scripts/kernel_breakdown.py --trace "$KT" --markers "$MT" --range bench.timed \
        --steps "${STEPS:-4}" > "$O/breakdown.txt" 2>&1
      head -30 "$O/breakdown.txt" ;;
    pmc_gemm)
      prof pmc_gemm 120 --kernel-trace \
        --pmc ${COUNTERS:-FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE} --output-format csv \
        -d "$O/pmc_gemm" -o run -- python3 -m mxk8s.validate.gemm --sizes "${SIZES:-8192}" \
        --variants "${VARIANTS:-26}" --iters 6 --rounds 2 --warmup-s 0.5 ;;
    contention)
      run contention 900 python3 -u scripts/contention_bench.py --cus "${CONT_CUS:-16,32,64}" --placement "${CONT_PLACE:-spread}" --gbps "${CONT_GBPS:-5,700}" ;;
    ddp_gloo2)
      run ddp_gloo2 600 env MXK_BENCH_BACKEND=gloo python3 -u bench.py --mode ddp --gpus 2 \
        --layers 2 --steps "${DDP_STEPS:-3}" --warmup 1 ${DDP_ARGS:-} ;;
    ddp_l2)
      run ddp_l2 300 python3 -u bench.py --mode ddp --layers 2 --steps "${DDP_STEPS:-3}" --warmup 1 ${DDP_ARGS:-} ;;
    validator_gloo2)
      run validator_gloo2 400 env MXK_BENCH_BACKEND=gloo python3 -u bench.py --gpus 2 --steps 10 \
        --warmup 2 --allreduce-sizes 1,16,256 --ab-sizes "" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
