#!/usr/bin/env bash
# TunableOp search over the Llama-3-8B step GEMMs, then untuned vs tuned timing.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
( while sleep 50; do date >> gpurun_out/heartbeat.txt; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=${TUNE_MS:-15}
export PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=${TUNE_IT:-10}
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 \
PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tuned%d.csv \
  timeout -k 10 900 python3 scripts/tune_gemms.py --tokens ${TOKENS:-8192} > gpurun_out/tune_gemms.log 2>&1
rc=$?; echo "tune rc=$rc"; grep RESULT gpurun_out/tune_gemms.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/tune_gemms.py --bench --tokens ${TOKENS:-8192} > gpurun_out/gemm_untuned.log 2>&1
rc=$?; echo "untuned rc=$rc"; [ $rc -eq 0 ] || exit $rc
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tuned%d.csv \
  timeout -k 10 300 python3 scripts/tune_gemms.py --bench --tokens ${TOKENS:-8192} > gpurun_out/gemm_tuned.log 2>&1
rc=$?; echo "tuned rc=$rc"
paste <(grep RESULT gpurun_out/gemm_untuned.log | python3 -c "import sys,json;[print(json.loads(l[7:])['gemm'], json.loads(l[7:])['tflops']) for l in sys.stdin]") \
      <(grep RESULT gpurun_out/gemm_tuned.log | python3 -c "import sys,json;[print(json.loads(l[7:])['tflops']) for l in sys.stdin]")
exit $rc
