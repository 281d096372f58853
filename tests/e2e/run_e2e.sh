#!/usr/bin/env bash
# End-to-end acceptance run of BASELINE.json configs 1-5 on a REAL MI355X node
# (root, network for the apt/kubeadm steps, 8 GPUs).  Not runnable in CI or on
# the gpurun boxes (no root, no kubelet); the CPU test suite checks this script
# with `bash -n` and `--plan`.
#
#   sudo tests/e2e/run_e2e.sh [--plan] [--skip-bootstrap] [--gpus 8] [--out e2e_results.jsonl]
#
# Every pass criterion is machine-checked (the reference's own check was
# reading `nvidia-smi` output after a fixed `sleep 15`, README.md:321-335):
#   1  node Ready, busybox pod Succeeded on the (untainted) control-plane node
#   2  allocatable amd.com/gpu == --gpus; hip-vector-add pod RESULT pass=true
#   3  gemm-validator pod: GEMM TFLOPS RESULT lines with pass=true
#   4  rccl-allreduce-8gpu pod: allreduce_summary at 1/2/4/8 GPUs, every point pass
#   5  llama3-8b-ddp-8gpu job: a DDP RESULT line (tokens/s, MFU)
set -euo pipefail
REPO=$(cd "$(dirname "$0")/../.." && pwd)
PLAN=0; SKIP_BOOT=0; GPUS=8; OUT=e2e_results.jsonl
while [ $# -gt 0 ]; do
  case "$1" in
    --plan) PLAN=1 ;;
    --skip-bootstrap) SKIP_BOOT=1 ;;
    --gpus) GPUS=$2; shift ;;
    --out) OUT=$2; shift ;;
    *) echo "unknown argument $1" >&2; exit 2 ;;
  esac
  shift
done

step() { echo "== $*"; }
run() { if [ $PLAN -eq 1 ]; then echo "+ $*"; else "$@"; fi; }
record() {   # record <config> <json>
  if [ $PLAN -eq 1 ]; then echo "+ record config $1"; return; fi
  python3 -c 'import json,sys; d=json.loads(sys.argv[2]); d["config"]=int(sys.argv[1]); print(json.dumps(d))' \
    "$1" "$2" >> "$OUT"
}
wait_pod() {   # wait_pod <name> <timeout>
  run kubectl wait "pod/$1" --for=jsonpath='{.status.phase}'=Succeeded --timeout="$2"
}
results_of() {   # RESULT lines of a pod's log
  if [ $PLAN -eq 1 ]; then echo "+ kubectl logs $1 | grep RESULT"; return; fi
  kubectl logs "$1" | sed -n 's/^RESULT //p'
}
check_all_pass() {   # stdin: RESULT json lines; fail unless every "pass" is true
  if [ $PLAN -eq 1 ]; then cat >/dev/null; return 0; fi
  python3 -c '
import json, sys
rs = [json.loads(l) for l in sys.stdin if l.strip()]
bad = [r for r in rs if r.get("pass") is False]
sys.exit(1 if not rs or bad else 0)'
}

[ $PLAN -eq 1 ] || : > "$OUT"

step "config 1: kubeadm single-node + Flannel, CPU-only busybox pod"
if [ $SKIP_BOOT -eq 0 ]; then
  run python3 -m mxk8s bootstrap
fi
run kubectl wait node --all --for=condition=Ready --timeout=600s
run kubectl -n kube-flannel rollout status ds/kube-flannel-ds --timeout=300s
run kubectl apply -f "$REPO/deploy/examples/busybox-smoke.yaml"
wait_pod busybox-smoke 300s
record 1 '{"test":"busybox","pass":true}'

step "config 2: device plugin, amd.com/gpu=1 pod runs rocminfo + HIP vectoradd"
run kubectl apply -f "$REPO/deploy/amd-gpu-stack.yaml"
run kubectl -n amd-gpu rollout status ds/amd-gpu-stack-device-plugin --timeout=300s
if [ $PLAN -eq 0 ]; then
  alloc=$(kubectl get nodes -o jsonpath='{.items[0].status.allocatable.amd\.com/gpu}')
  [ "$alloc" = "$GPUS" ] || { echo "allocatable amd.com/gpu=$alloc, expected $GPUS" >&2; exit 1; }
  record 2 "{\"test\":\"allocatable\",\"amd.com/gpu\":$alloc,\"pass\":true}"
fi
run kubectl apply -f "$REPO/deploy/examples/hip-vector-add.yaml"
wait_pod hip-vector-add 300s
# every RESULT line passes AND the pod sees exactly its 1 allocated gfx950
# GPU / render node (BASELINE.md:37)
results_of hip-vector-add | run env PYTHONPATH="$REPO" python3 -m mxk8s.validate.isolation --gpus 1 --arch gfx950
record 2 '{"test":"hip-vector-add","pass":true,"isolation":true}'

step "config 3: validator pod amd.com/gpu=1, bf16 MFMA GEMM"
run kubectl apply -f "$REPO/deploy/examples/gemm-validator.yaml"
wait_pod gemm-validator 1800s
results_of gemm-validator | check_all_pass
if [ $PLAN -eq 0 ]; then results_of gemm-validator | while read -r l; do record 3 "$l"; done; fi

step "config 4: amd.com/gpu=8 RCCL all-reduce, 1/2/4/8 bus-bw curve"
run kubectl apply -f "$REPO/deploy/examples/rccl-allreduce-8gpu.yaml"
wait_pod rccl-allreduce 3600s
results_of rccl-allreduce | check_all_pass
if [ $PLAN -eq 0 ]; then
  results_of rccl-allreduce | grep '_summary' | while read -r l; do record 4 "$l"; done
fi

step "config 5: PyTorch-ROCm DDP Llama-3-8B training step on amd.com/gpu=8"
run kubectl apply -f "$REPO/deploy/examples/llama3-8b-ddp-8gpu.yaml"
run kubectl wait job/llama3-8b-ddp --for=condition=complete --timeout=7200s
if [ $PLAN -eq 0 ]; then
  kubectl logs job/llama3-8b-ddp | grep '^{' | tail -1 | while read -r l; do record 5 "$l"; done
fi

step "done: results in $OUT"
run python3 -m mxk8s doctor gpu
