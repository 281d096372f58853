set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r4abl; mkdir -p $O
export PYTHONPATH=. MXK_KERNELS_LIB=$PWD/mxk8s/_lib/libmxkernels_exp.so
timeout -k 10 300 python3 -u -m mxk8s.validate.gemm --sizes 8192 --shapes 4096x4096x16384 --variants 26,54,47,52,53,10,48,49,50,51 --iters 96 --rounds 12 > $O/abl.log 2>&1
rc=$?
grep RESULT $O/abl.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l.split('RESULT ', 1)[1]); print(d['kernel'], d['M'], d['K'], round(d['tflops_median'], 1), round(d['median_ms'],4))"
exit $rc
