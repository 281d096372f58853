#!/usr/bin/env bash
# One GPU call: GPU tests, the validator bench (default schedule), PMC
# counters + kernel stats of the default GEMM, summaries into gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
mkdir -p gpurun_out
export PYTHONPATH=$R${PYTHONPATH:+:$PYTHONPATH}
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 100 --warmup 50 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
VARIANTS=5 SIZES=${SIZES:-8192} bash scripts/gpu/gemm_pmc.sh
rc=$?; [ $rc -eq 0 ] || exit $rc
python3 scripts/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 > gpurun_out/pmc_summary.txt 2>&1
echo "summary rc=$?"; cat gpurun_out/pmc_summary.txt
