#!/usr/bin/env bash
# GEMM L2 / tile-order probe: schedule 26 against the tile-map (41-43) and
# K-rotation (44) A/B records, time + FETCH_SIZE per size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
O=$R/${1:-gpurun_out/r4map}
V=${VARIANTS:-26,41,42,43}
mkdir -p $O
export PYTHONPATH=$R TMPDIR=/tmp MXK_KERNELS_LIB=$R/mxk8s/_lib/libmxkernels_exp.so
timeout -k 10 400 python3 -u -m mxk8s.validate.gemm --sizes 8192,4096,16384 --shapes 4096x4096x16384 --variants $V --iters 96 --rounds 12 > $O/map_ab.log 2>&1 && \
( cd /tmp && timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o run -- python3 -m mxk8s.validate.gemm --sizes 8192,16384 --shapes 4096x4096x16384 --variants $V --iters 6 --rounds 2 --warmup-s 0.5 > $O/pmc.log 2>&1 )
rc=$?
grep -h RESULT $O/map_ab.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l.split('RESULT ', 1)[1]); print(d['kernel'], d['M'], d['N'], d['K'], d['lda'], round(d['tflops_median'], 1))"
python3 scripts/pmc_by_grid.py $O/pmc --filter gemm
exit $rc
