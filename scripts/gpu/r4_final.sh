# Round-4 closing pass: attention backward variant 5 check + timing, PMC of
# the default GEMM against hipBLASLt, then the full GPU tier, smoke, the
# driver's bench command, the DDP step and its kernel profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=${1:-gpurun_out/r4final}; mkdir -p $O
export PYTHONPATH=.
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_attention.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_attn.log 2>&1 || { tail -5 $O/pytest_attn.log; exit 1; }
tail -1 $O/pytest_attn.log
BATCH=8 timeout -k 10 300 python3 -u scripts/attn_mxk_bench.py > $O/attn_b8.log 2>&1 || exit 1
grep RESULT $O/attn_b8.log | head -20
VARIANTS=52 SIZES=8192,16384 bash scripts/gpu/pass.sh $O pmc_gemm || exit 1
bash scripts/gpu/pass.sh $O pytest smoke bench bench_ddp prof_ddp
