#!/usr/bin/env bash
# Fused RoPE (ABVAR, default MXK_FUSED_ROPE_BWD; =1 the default) against the unfused
# chain (=0): the attention GPU tests, then alternating DDP-step runs of the
# Llama-3-8B bench (separate processes, same box).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=${1:-gpurun_out/rope_ab}
mkdir -p "$O"
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_attention.py -x -q --timeout 120 --timeout-method thread > "$O/test.log" 2>&1
rc=$?; echo "attention tests rc=$rc: $(tail -1 "$O/test.log")"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for f in 1 0; do
    env ${ABVAR:-MXK_FUSED_ROPE_BWD}=$f timeout -k 10 400 python3 -u bench.py --mode ddp --steps 8 --warmup 2 > "$O/ddp_f${f}_$r.out" 2> "$O/ddp_f${f}_$r.err"
    rc=$?; echo "fused=$f run $r rc=$rc: $(python3 -c "import json,sys; d=json.loads(open('$O/ddp_f${f}_$r.out').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['losses'])" 2>&1)"
    [ $rc -eq 0 ] || exit $rc
  done
done
