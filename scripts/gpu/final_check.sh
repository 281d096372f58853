#!/usr/bin/env bash
# End-of-round GPU pass: the full GPU test tier, the driver's smoke(), the
# headline bench at the driver's arguments, the DDP step, and the DDP step's
# steady-state kernel breakdown (kernel trace bounded by the bench.timed roctx
# range).  Every step has its own time limit; the first failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
O=${1:-gpurun_out/final}
mkdir -p "$O"
export PYTHONPATH=$R${PYTHONPATH:+:$PYTHONPATH}
step() {   # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.out" 2> "$O/$name.err"
  local rc=$?
  echo "$name rc=$rc"
  tail -2 "$O/$name.out"
  [ $rc -eq 0 ] || exit $rc
}
step pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench_driver_args 300 python3 bench.py --steps 20 --warmup 5
step bench_ddp 400 python3 bench.py --mode ddp --steps 10 --warmup 3
