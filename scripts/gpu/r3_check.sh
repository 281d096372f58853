#!/usr/bin/env bash
# Round-3 GPU check: ring/variant correctness sweep, the fused-MLP / split-tail
# GPU tests, GEMM schedule A/B, and a short Llama-3-8B DDP step on the new
# forward path.  Every GPU step has its own time limit; the first failure ends
# the script.
set -o pipefail
OUT=${1:-gpurun_out/r3d}
mkdir -p "$OUT"
export PYTHONPATH=.
EXP=mxk8s/_lib/libmxkernels_exp.so
MXK_KERNELS_LIB=$EXP timeout -k 10 150 python -u scripts/gpu/ring_check.py 26,29,30 > "$OUT/ring_check.log" 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp_fused.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_mlp.log" 2>&1 && \
MXK_KERNELS_LIB=$EXP timeout -k 10 300 python -u -m mxk8s.validate.gemm --sizes 8192,4096,16384 --variants 26,29,30 --iters 96 --rounds 12 > "$OUT/gemm_ab.log" 2>&1 && \
timeout -k 10 420 python -u bench.py --mode ddp --steps 6 --warmup 2 > "$OUT/bench_ddp.log" 2>&1
