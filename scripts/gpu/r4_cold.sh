# GEMM A/B with the operands cache-warm (back-to-back launches of one pair)
# and HBM-cold (4 pairs cycled, beyond the 256 MB Infinity Cache) on the
# Llama-3-8B forward shapes at 16k tokens and 8192^3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/r4cold; mkdir -p $O
export PYTHONPATH=.
for c in 1 4; do
  timeout -k 10 300 python3 -u -m mxk8s.validate.gemm --sizes 8192 --shapes 16384x4096x4096,16384x6144x4096,16384x4096x14336 \
    --variants ${VARIANTS:-26,52,56} --iters 48 --rounds 12 --cold $c > $O/cold$c.log 2>&1 || exit $?
done
for c in 1 4; do
  grep RESULT $O/cold$c.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l.split('RESULT ', 1)[1]); print('cold', d['cold_pairs'], d['kernel'], d['M'], d['N'], d['K'], round(d['tflops_median'], 1))"
done
