#!/usr/bin/env bash
# Kernel-level profile of the Llama-3-8B DDP step (world size 1).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$R${PYTHONPATH:+:$PYTHONPATH}
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_ddp -o run -- \
  python3 $R/bench.py --mode ddp --steps ${STEPS:-4} --warmup 2 > $R/gpurun_out/prof_ddp.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -2 $R/gpurun_out/prof_ddp.log; exit $rc
