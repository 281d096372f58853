#!/usr/bin/env bash
# Run the native validator binaries + the Python validator on one MI355X.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 120 ./bin/mx-vector-add --n 50000 > gpurun_out/vadd.log 2>&1; rc=$?; echo "vadd rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 ./bin/mx-gemm-bench --sizes 4096,8192 --iters 30 --warmup-ms 1000 > gpurun_out/gemm_bench.log 2>&1; rc=$?; echo "gemm rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 ./bin/mx-allreduce-perf -b 8 -e 1G -f 4 --scaling 1,2 > gpurun_out/rccl.log 2>&1; rc=$?; echo "rccl rc=$rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python3 -m mxk8s.validate --tests rocminfo,vectoradd,gemm,rccl --gpus 1 --gemm-sizes 8192 --rccl-max-bytes 268435456 > gpurun_out/validate.log 2> gpurun_out/validate.err; rc=$?; echo "validate rc=$rc"
cat gpurun_out/vadd.log gpurun_out/gemm_bench.log; grep RESULT gpurun_out/rccl.log | tail -4; grep RESULT gpurun_out/validate.log | tail -3
exit $rc
