"""mxk8s — an MI355X-native single-node Kubernetes GPU stack.

Capabilities mirror the NVIDIA recipe mysticrenji/kubernetes-with-nvidia-gpu
(/root/reference/README.md), re-designed for AMD Instinct MI355X (gfx950):

* host bring-up (``mxk8s.bootstrap``): swap/modules/sysctl, amdgpu+ROCm gate,
  containerd with CDI, kubeadm v1.34 + Flannel, control-plane untaint
* ROCm CDI spec + ``amd.com/gpu`` device plugin (``mxk8s.deviceplugin``) on
  the native discovery core ``libmxnode`` (``native/libmxnode``)
* node labeller (``mxk8s.labeller``) and amd-smi Prometheus exporter
  (``mxk8s.exporter``) replacing GFD and DCGM
* Helm chart ``charts/amd-gpu-stack`` + offline renderer (``mxk8s.chart``)
* validators (``mxk8s.validate``): HIP vectoradd, CDNA4 bf16 MFMA GEMM,
  RCCL all-reduce over xGMI, Llama-3-8B DDP training step
* ``mxk8s doctor`` troubleshooting
"""

__version__ = "0.1.0"

RESOURCE_NAME = "amd.com/gpu"
NAMESPACE = "amd-gpu"
RELEASE_NAME = "amd-gpu-stack"
