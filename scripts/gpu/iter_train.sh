#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 scripts/attn_bench.py > gpurun_out/attn_bench.log 2>&1; rc=$?
echo "attn rc=$rc"; cat gpurun_out/attn_bench.log | grep -v amdgpu.ids; [ $rc -le 1 ] || exit $rc
timeout -k 10 900 python3 bench.py --mode ddp --steps 5 --warmup 2 > gpurun_out/ddp8b.log 2>&1; rc=$?
echo "ddp rc=$rc"; tail -1 gpurun_out/ddp8b.log
exit $rc
