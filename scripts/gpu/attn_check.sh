#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
timeout -k 10 300 python3 -m pytest tests/test_gpu_attention.py -x -q > gpurun_out/attn_test.log 2>&1
rc=$?; echo "attn test rc=$rc"; tail -25 gpurun_out/attn_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/attn_mxk_bench.py > gpurun_out/attn_bench.log 2>&1 && BATCH=8 timeout -k 10 300 python3 scripts/attn_mxk_bench.py >> gpurun_out/attn_bench.log 2>&1
rc=$?; echo "attn bench rc=$rc"; grep RESULT gpurun_out/attn_bench.log; exit $rc
