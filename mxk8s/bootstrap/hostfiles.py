"""Host configuration files written by ``mxk8s bootstrap`` — one source of truth.

Each function returns file content; ``phases.py`` decides where and when.
Reference steps reproduced (MI355X-first additions noted):

* modules-load.d/k8s.conf: overlay, br_netfilter      (README.md:37-43)
* sysctl.d/k8s.conf: bridge-nf-call-ip(6)tables, ip_forward (README.md:49-55)
  + sysctl.d/99-amd-gpu.conf: kernel.numa_balancing=0 (AMD Instinct tuning)
* fstab with swap entries commented                    (README.md:28-29)
* containerd config: SystemdCgroup = true              (README.md:121-123)
  + CDI enabled (replaces nvidia-ctk runtime configure, README.md:145-149)
* kubeadm-config.yaml: podSubnet 10.244.0.0/16, cgroupDriver systemd,
  Kubernetes v1.34                                     (README.md:164-202)
"""
from __future__ import annotations

import re

import yaml

K8S_MINOR = "v1.34"
K8S_VERSION = "v1.34.1"
POD_CIDR = "10.244.0.0/16"
HELM_VERSION = "v3.19.0"
CRI_SOCKET = "unix:///run/containerd/containerd.sock"
CDI_DIRS = ["/etc/cdi", "/var/run/cdi"]
CDI_SPEC_PATH = "/etc/cdi/amd.com-gpu.json"
PHASE_FILE = "/var/lib/mxk8s/phase"


def modules_load_conf() -> str:
    return "# mxk8s: kernel modules for containerd overlayfs + kube-proxy/flannel bridging\noverlay\nbr_netfilter\n"


def sysctl_k8s_conf() -> str:
    return ("# mxk8s: Kubernetes networking\n"
            "net.bridge.bridge-nf-call-iptables  = 1\n"
            "net.bridge.bridge-nf-call-ip6tables = 1\n"
            "net.ipv4.ip_forward                 = 1\n")


def sysctl_amd_gpu_conf() -> str:
    # AMD Instinct guidance: automatic NUMA balancing migrates pages under
    # running GPU jobs and hurts host<->GPU transfers.
    return "# mxk8s: AMD Instinct MI355X host tuning\nkernel.numa_balancing = 0\n"


def comment_swap(fstab: str) -> str:
    """Comment out every active swap entry (same effect as README.md:29's sed)."""
    out = []
    for line in fstab.splitlines(keepends=True):
        fields = line.split()
        if line.lstrip().startswith("#") or len(fields) < 3:
            out.append(line)
        elif fields[2] == "swap" or " swap " in f" {line} ":
            out.append("#" + line)
        else:
            out.append(line)
    return "".join(out)


# --------------------------------------------------------------------------
# containerd: SystemdCgroup + CDI, for both config schema versions
# --------------------------------------------------------------------------

def containerd_config_version(text: str) -> int:
    m = re.search(r"^\s*version\s*=\s*(\d+)", text, re.M)
    return int(m.group(1)) if m else 1


def _set_in_table(text: str, table: str, key: str, value: str) -> str:
    """Set `key = value` inside [table] (create table / key if missing)."""
    hdr = re.compile(r"^\s*\[" + re.escape(table) + r"\]\s*$", re.M)
    m = hdr.search(text)
    if not m:
        sep = "" if text.endswith("\n") or not text else "\n"
        return f"{text}{sep}\n[{table}]\n  {key} = {value}\n"
    start = m.end()
    nxt = re.compile(r"^\s*\[", re.M).search(text, start)
    end = nxt.start() if nxt else len(text)
    body = text[start:end]
    kre = re.compile(r"^(\s*)" + re.escape(key) + r"\s*=.*$", re.M)
    if kre.search(body):
        body = kre.sub(lambda mm: f"{mm.group(1)}{key} = {value}", body, count=1)
    else:
        indent = "  "
        first = re.search(r"^(\s+)\S", body, re.M)
        if first:
            indent = first.group(1).replace("\n", "")
        body = f"\n{indent}{key} = {value}" + body
    return text[:start] + body + text[end:]


def configure_containerd(text: str) -> str:
    """Apply SystemdCgroup = true and enable CDI to a `containerd config
    default` dump (containerd 1.7: config version 2; containerd 2.x: 3)."""
    ver = containerd_config_version(text)
    dirs = "[" + ", ".join(f'"{d}"' for d in CDI_DIRS) + "]"
    if ver >= 3:
        runc = 'plugins."io.containerd.cri.v1.runtime".containerd.runtimes.runc.options'
        cri = 'plugins."io.containerd.cri.v1.runtime"'
    else:
        runc = 'plugins."io.containerd.grpc.v1.cri".containerd.runtimes.runc.options'
        cri = 'plugins."io.containerd.grpc.v1.cri"'
    text = _set_in_table(text, runc, "SystemdCgroup", "true")
    text = _set_in_table(text, cri, "enable_cdi", "true")
    text = _set_in_table(text, cri, "cdi_spec_dirs", dirs)
    return text


def minimal_containerd_config(version: int = 2) -> str:
    """What `containerd config default` would start from when containerd is not
    installed (dry runs / tests)."""
    if version >= 3:
        return ('version = 3\n\n[plugins]\n\n  [plugins."io.containerd.cri.v1.runtime"]\n'
                '    enable_cdi = false\n\n'
                '  [plugins."io.containerd.cri.v1.runtime".containerd.runtimes.runc.options]\n'
                '    SystemdCgroup = false\n')
    return ('version = 2\n\n[plugins]\n\n  [plugins."io.containerd.grpc.v1.cri"]\n'
            '    enable_cdi = false\n    sandbox_image = "registry.k8s.io/pause:3.10"\n\n'
            '  [plugins."io.containerd.grpc.v1.cri".containerd.runtimes.runc.options]\n'
            '    SystemdCgroup = false\n')


# --------------------------------------------------------------------------
# kubeadm
# --------------------------------------------------------------------------

def kubeadm_config(node_name: str = "", advertise_address: str = "",
                   k8s_version: str = K8S_VERSION, pod_cidr: str = POD_CIDR) -> str:
    init = {"apiVersion": "kubeadm.k8s.io/v1beta4", "kind": "InitConfiguration",
            "nodeRegistration": {"criSocket": CRI_SOCKET,
                                 # untaint up front: single-node cluster (the
                                 # reference never removed the taint)
                                 "taints": []}}
    if node_name:
        init["nodeRegistration"]["name"] = node_name
    if advertise_address:
        init["localAPIEndpoint"] = {"advertiseAddress": advertise_address, "bindPort": 6443}
    cluster = {"apiVersion": "kubeadm.k8s.io/v1beta4", "kind": "ClusterConfiguration",
               "kubernetesVersion": k8s_version,
               "networking": {"podSubnet": pod_cidr, "serviceSubnet": "10.96.0.0/12"}}
    kubelet = {"apiVersion": "kubelet.config.k8s.io/v1beta1", "kind": "KubeletConfiguration",
               "cgroupDriver": "systemd",
               # Topology Manager uses the NUMA nodes our device plugin reports
               "topologyManagerPolicy": "best-effort"}
    return "---\n".join(yaml.safe_dump(d, sort_keys=False) for d in (init, cluster, kubelet))


def k8s_minor(version: str) -> str:
    """v1.34.1 -> v1.34 (the pkgs.k8s.io repository path)."""
    return ".".join(version.split(".")[:2])


def kubernetes_apt_source(minor: str = K8S_MINOR) -> str:
    return (f"deb [signed-by=/etc/apt/keyrings/kubernetes-apt-keyring.gpg] "
            f"https://pkgs.k8s.io/core:/stable:/{minor}/deb/ /\n")
