#!/usr/bin/env bash
# Same-box DDP step A/B: production fused up-projection vs the persistent
# form (experiments library, MXK_W13_SCHED=3), alternating processes.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=${1:-gpurun_out/w13_step}
mkdir -p "$O"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --mode ddp --steps 8 --warmup 3 > "$O/base_$i.out" 2> "$O/base_$i.err"
  rc=$?; echo "base $i rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$O/base_$i.out")"; [ $rc -eq 0 ] || exit $rc
  MXK_KERNELS_LIB=$PWD/mxk8s/_lib/libmxkernels_exp.so MXK_W13_SCHED=3 timeout -k 10 300 python3 bench.py --mode ddp --steps 8 --warmup 3 > "$O/w13p_$i.out" 2> "$O/w13p_$i.err"
  rc=$?; echo "w13p $i rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$O/w13p_$i.out")"; [ $rc -eq 0 ] || exit $rc
done
