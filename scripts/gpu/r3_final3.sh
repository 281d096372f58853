#!/usr/bin/env bash
# Last round-3 pass on the final tree: the GPU tier on the production
# library, the A/B-record kernels (trickle-store GEMMs, every TN schedule,
# attention forward 5-9) on the experiments library, smoke(), the headline
# bench at the driver's arguments and the DDP step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
OUT=${1:-gpurun_out/r3final3}
mkdir -p "$OUT"
export PYTHONPATH=.
step() {
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc"; tail -1 "$OUT/$name.out"
  [ $rc -eq 0 ] || exit $rc
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step pytest_exp 600 env MXK_KERNELS_LIB=$PWD/mxk8s/_lib/libmxkernels_exp.so python -u -m pytest tests -m gpu -k "attn_fwd or schedule or trickle" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench_driver_args 300 python bench.py --steps 20 --warmup 5
step bench_ddp 400 python bench.py --mode ddp --steps 10 --warmup 3
