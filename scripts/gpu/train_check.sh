#!/usr/bin/env bash
# GPU tests + smoke + full Llama-3-8B DDP step at world size 1.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 900 python3 bench.py --mode ddp --steps ${STEPS:-5} --warmup 2 > gpurun_out/ddp8b.log 2>&1; rc=$?
echo "ddp rc=$rc"; tail -3 gpurun_out/ddp8b.log
exit $rc
