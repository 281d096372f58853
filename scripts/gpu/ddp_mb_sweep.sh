#!/usr/bin/env bash
# Llama-3-8B DDP step at world size 1 for several micro-batch sizes.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -m pytest tests/test_gpu_train.py -x -q > gpurun_out/pytest_train.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_train.log; [ $rc -eq 0 ] || exit $rc
for mb in ${MBS:-1 2 4}; do
  timeout -k 10 600 python3 bench.py --mode ddp --steps 6 --warmup 2 --micro-batch $mb > gpurun_out/ddp_mb$mb.log 2>&1; rc=$?
  echo "mb=$mb rc=$rc"; tail -1 gpurun_out/ddp_mb$mb.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
done
