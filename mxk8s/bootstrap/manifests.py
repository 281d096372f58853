"""Workload manifests for the five BASELINE.json configs, generated from one
place and written to ``deploy/examples/`` (``python -m mxk8s.bootstrap.manifests``).

Every pod tolerates the control-plane taint (the reference's smoke pod at
README.md:303-318 had no toleration and would stay Pending on a stock kubeadm
node) and GPU pods mount a memory-backed /dev/shm for RCCL.

  config 1  busybox-smoke.yaml          CPU-only plumbing check
  config 2  hip-vector-add.yaml         amd.com/gpu: 1 -> rocminfo + HIP vectoradd (README.md:298-335)
  config 3  gemm-validator.yaml         amd.com/gpu: 1 -> CDNA4 bf16 MFMA GEMM
  config 4  rccl-allreduce-8gpu.yaml    amd.com/gpu: 8 -> RCCL all-reduce bus-bw sweep over xGMI
  config 5  llama3-8b-ddp-8gpu.yaml     amd.com/gpu: 8 -> PyTorch-ROCm DDP Llama-3-8B step
"""
from __future__ import annotations

import os
import sys

import yaml

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
IMAGE = "ghcr.io/mxk8s/mxk8s:0.1.0"
RESOURCE = "amd.com/gpu"

TOLERATIONS = [
    {"key": "node-role.kubernetes.io/control-plane", "operator": "Exists", "effect": "NoSchedule"},
    {"key": RESOURCE, "operator": "Exists", "effect": "NoSchedule"},
]


def _gpu_container(name: str, command: list, gpus: int, extra_env=None, cpu="4", mem="32Gi") -> dict:
    env = [{"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"}] + (extra_env or [])
    return {"name": name, "image": IMAGE, "imagePullPolicy": "IfNotPresent",
            "command": command, "env": env,
            "resources": {"limits": {RESOURCE: gpus},
                          "requests": {RESOURCE: gpus, "cpu": cpu, "memory": mem}},
            "volumeMounts": [{"name": "dshm", "mountPath": "/dev/shm"}]}


def _dshm(size: str) -> dict:
    return {"name": "dshm", "emptyDir": {"medium": "Memory", "sizeLimit": size}}


def busybox_smoke() -> dict:
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": "busybox-smoke", "labels": {"app": "mxk8s-smoke"}},
            "spec": {"restartPolicy": "Never", "tolerations": TOLERATIONS,
                     "containers": [{"name": "busybox", "image": "busybox:1.36",
                                     "command": ["sh", "-c",
                                                 "nslookup kubernetes.default.svc.cluster.local >/dev/null 2>&1 "
                                                 "&& dns=true || dns=false; "
                                                 "echo RESULT '{\"config\":1,\"pass\":true,\"dns\":'$dns'}'"]}]}}


def hip_vector_add() -> dict:
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": "hip-vector-add", "labels": {"app": "mxk8s-smoke"}},
            "spec": {"restartPolicy": "OnFailure", "tolerations": TOLERATIONS,
                     "containers": [_gpu_container(
                         "hip-vector-add",
                         ["sh", "-c", "rocminfo | grep -E '^\\s+Name:\\s+gfx' ; ls -l /dev/dri ; "
                                      "env | grep '^AMD_GPU_' ; "
                                      "exec /opt/mxk8s/bin/mx-vector-add --n 50000 --check "
                                      "--expect-gpus 1 --expect-arch gfx950"],
                         1, cpu="1", mem="2Gi")],
                     "volumes": [_dshm("1Gi")]}}


def gemm_validator() -> dict:
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": "gemm-validator", "labels": {"app": "mxk8s-validator"}},
            "spec": {"restartPolicy": "OnFailure", "tolerations": TOLERATIONS,
                     "containers": [_gpu_container(
                         "gemm", ["python3", "-m", "mxk8s.validate", "--tests=rocminfo,gemm",
                                  "--gpus=1", "--gemm-sizes=4096,8192,16384", "--profile"], 1)],
                     "volumes": [_dshm("8Gi")]}}


def _rccl_env() -> list:
    from ..parallel import rccl_env
    return [{"name": k, "value": v} for k, v in sorted(rccl_env.resolve("xgmi-node").items())]


def rccl_allreduce_8gpu() -> dict:
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": "rccl-allreduce", "labels": {"app": "mxk8s-validator"}},
            "spec": {"restartPolicy": "OnFailure", "tolerations": TOLERATIONS,
                     # all 8 GPUs in ONE pod: RCCL P2P/IPC needs one IPC namespace
                     "containers": [_gpu_container(
                         "rccl", ["python3", "-m", "mxk8s.validate", "--tests=rccl", "--gpus=8",
                                  "--rccl-min-bytes=8", "--rccl-max-bytes=8589934592",
                                  "--rccl-scaling=1,2,4,8"], 8, extra_env=_rccl_env(),
                         cpu="16", mem="128Gi")],
                     "volumes": [_dshm("64Gi")]}}


def llama3_ddp_8gpu() -> dict:
    return {"apiVersion": "batch/v1", "kind": "Job",
            "metadata": {"name": "llama3-8b-ddp", "labels": {"app": "mxk8s-train"}},
            "spec": {"backoffLimit": 1, "template": {
                "metadata": {"labels": {"app": "mxk8s-train"}},
                "spec": {"restartPolicy": "Never", "tolerations": TOLERATIONS,
                         "containers": [_gpu_container(
                             "train",
                             ["python3", "-m", "torch.distributed.run", "--standalone",
                              "--nproc-per-node=8", "/opt/mxk8s/bench.py", "--mode=ddp",
                              "--gpus=8", "--steps=10", "--warmup=3", "--seq-len=2048"],
                             8, extra_env=_rccl_env(), cpu="64", mem="512Gi")],
                         "volumes": [_dshm("64Gi")]}}}}


EXAMPLES = {
    "busybox-smoke.yaml": busybox_smoke,
    "hip-vector-add.yaml": hip_vector_add,
    "gemm-validator.yaml": gemm_validator,
    "rccl-allreduce-8gpu.yaml": rccl_allreduce_8gpu,
    "llama3-8b-ddp-8gpu.yaml": llama3_ddp_8gpu,
}

HEADER = "# Generated by `python -m mxk8s.bootstrap.manifests` — do not edit by hand.\n"


def render_examples() -> dict[str, str]:
    return {n: HEADER + yaml.safe_dump(fn(), sort_keys=False) for n, fn in EXAMPLES.items()}


def write_deploy(repo: str = REPO) -> list[str]:
    """Regenerate deploy/: examples, kubeadm config, rendered chart."""
    from . import hostfiles as hf
    from ..chart import render as chart
    written = []
    ex = os.path.join(repo, "deploy", "examples")
    os.makedirs(ex, exist_ok=True)
    for n, text in render_examples().items():
        with open(os.path.join(ex, n), "w") as f:
            f.write(text)
        written.append(os.path.join("deploy", "examples", n))
    with open(os.path.join(repo, "deploy", "kubeadm-config.yaml"), "w") as f:
        f.write(HEADER + hf.kubeadm_config())
    written.append("deploy/kubeadm-config.yaml")
    with open(os.path.join(repo, "deploy", "amd-gpu-stack.yaml"), "w") as f:
        f.write("# Rendered from charts/amd-gpu-stack with default values "
                "(python -m mxk8s.chart.render).\n" + chart.to_stream(chart.render()))
    written.append("deploy/amd-gpu-stack.yaml")
    return written


if __name__ == "__main__":
    for p in write_deploy():
        print(p)
    sys.exit(0)
