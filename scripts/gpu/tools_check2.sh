#!/usr/bin/env bash
# Collective sweep (every op, n=1) + validator with the rocprofv3 counter pass.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
mkdir -p gpurun_out
export PYTHONPATH=$R${PYTHONPATH:+:$PYTHONPATH}
export TMPDIR=/tmp
timeout -k 10 300 bin/mx-allreduce-perf -b 8 -e 1G -f 4 --op all --dtype bf16 > gpurun_out/coll_all.log 2>&1
rc=$?; echo "coll rc=$rc"; grep -E "summary|FAIL" gpurun_out/coll_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -m mxk8s.validate --tests gemm --gemm-sizes 8192 --profile \
    --profile-dir $R/gpurun_out/val_pmc > gpurun_out/validate_profile.log 2>&1
rc=$?; echo "validate rc=$rc"; grep RESULT gpurun_out/validate_profile.log | cut -c1-400; exit $rc
