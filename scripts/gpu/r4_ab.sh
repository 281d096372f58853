# Round-4 GEMM default decision: the three protocol sizes, schedules 26 (round-3
# default), 47 / 52 (one-barrier w4k), 54 / 55 (staggered rounds), hipBLASLt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r4ab; mkdir -p $O
export PYTHONPATH=. MXK_KERNELS_LIB=$PWD/mxk8s/_lib/libmxkernels_exp.so
timeout -k 10 420 python3 -u -m mxk8s.validate.gemm --sizes 8192,4096,16384 --variants ${VARIANTS:-26,47,52,54,55} \
  --iters 64 --rounds 16 > $O/ab.log 2>&1
rc=$?
grep RESULT $O/ab.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l.split('RESULT ', 1)[1]); print(d['kernel'], d['M'], d['K'], round(d['tflops_median'], 1), round(d['median_ms'],4))"
exit $rc
