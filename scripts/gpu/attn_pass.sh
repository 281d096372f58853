set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r5_attn1
export PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_attention.py -k "v6 or variants or onepass" > gpurun_out/r5_attn1/pytest.out 2>&1; rc=$?; echo pytest rc=$rc; tail -5 gpurun_out/r5_attn1/pytest.out; [ $rc -eq 0 ] || exit $rc
BATCH=8 timeout -k 10 300 python3 -u scripts/attn_mxk_bench.py > gpurun_out/r5_attn1/bench_b8.out 2>&1; rc=$?; echo bench rc=$rc; cat gpurun_out/r5_attn1/bench_b8.out | grep RESULT
