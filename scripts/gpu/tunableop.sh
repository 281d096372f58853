#!/usr/bin/env bash
# Tune the Llama-3-8B step's GEMMs with PyTorch TunableOp (hipBLASLt + rocBLAS
# solution search), then re-run the step with the tuned table only.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export PYTORCH_TUNABLEOP_ENABLED=1
export PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tunableop_results%d.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=${TUNE_MS:-60}
export PYTORCH_TUNABLEOP_VERBOSE=1
PYTORCH_TUNABLEOP_TUNING=1 timeout -k 10 900 python3 bench.py --mode ddp --steps 2 --warmup 1 > gpurun_out/tune.log 2>&1
rc=$?; echo "tune rc=$rc"; tail -1 gpurun_out/tune.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
ls -la gpurun_out/tunableop_results*.csv
PYTORCH_TUNABLEOP_TUNING=0 timeout -k 10 600 python3 bench.py --mode ddp --steps 6 --warmup 2 > gpurun_out/tuned_run.log 2>&1
rc=$?; echo "tuned run rc=$rc"; tail -1 gpurun_out/tuned_run.log | cut -c1-400; exit $rc
