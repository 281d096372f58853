#!/usr/bin/env bash
# Llama-3-8B step (mb 4): default hipBLASLt picks vs the TunableOp table.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py --mode ddp --steps 6 --warmup 2 --no-tuned-gemms > gpurun_out/ddp_untuned.log 2>&1; rc=$?
echo "untuned rc=$rc"; tail -1 gpurun_out/ddp_untuned.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('tuned_gemms'))"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 bench.py --mode ddp --steps 6 --warmup 2 > gpurun_out/ddp_tuned.log 2>&1; rc=$?
echo "tuned rc=$rc"; tail -1 gpurun_out/ddp_tuned.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('tuned_gemms'))"; exit $rc
