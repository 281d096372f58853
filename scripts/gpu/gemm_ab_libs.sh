#!/usr/bin/env bash
# A/B alternative kernel builds (build/ab/*.so) against the in-tree library on
# the default GEMM schedule.  Each build runs in its own process.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/ab
for lib in mxk8s/_lib/libmxkernels.so build/ab/*.so; do
  name=$(basename "$lib" .so)
  MXK_KERNELS_LIB="$PWD/$lib" timeout -k 10 240 python3 -m mxk8s.validate.gemm \
      --sizes ${SIZES:-8192,4096} --iters 60 --rounds 6 > gpurun_out/ab/$name.log 2>&1 || { echo "$name failed"; exit 1; }
  grep RESULT gpurun_out/ab/$name.log | python3 -c "
import sys, json
for l in sys.stdin:
    r = json.loads(l[7:]); print(f\"$name {r['kernel']:14s} {r['M']:6d} {r['tflops_median']:8.1f} TF (best {r['tflops_best']:.1f})\")
"
done
