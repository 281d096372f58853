#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
timeout -k 10 400 python3 scripts/gemm_layouts_bench.py > gpurun_out/gemm_layouts.log 2>&1
rc=$?; echo "rc=$rc"; grep -E "RESULT|Error|wrong" gpurun_out/gemm_layouts.log | cut -c1-260; tail -3 gpurun_out/gemm_layouts.log; exit $rc
