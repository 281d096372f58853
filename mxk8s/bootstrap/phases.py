"""Idempotent, resumable, phase-gated host bring-up (``mxk8s bootstrap``).

The reference is a manual runbook (/root/reference/README.md:13-335) with a
reboot in the middle (README.md:70-74), a "do not proceed" gate (:84), a fixed
``sleep 15`` (:326) and a control-plane taint it never removes.  Here every
step is a phase with a completion marker in /var/lib/mxk8s/phase, so a rerun
after the reboot (or after any failure) resumes where it stopped:

  preflight     root, Ubuntu release, CPU/memory/disk, offline-capable          README.md:5-9
  prep          swap off, overlay/br_netfilter, sysctls (+ numa_balancing=0)   README.md:13-56
  driver-check  amdgpu loaded, /dev/kfd, gfx950 GPUs via libmxnode, iommu=pt   README.md:60-84
  runtime       containerd, SystemdCgroup=true, CDI enabled                    README.md:88-124,151-155
  cdi           /etc/cdi/amd.com-gpu.json from mx-cdi-gen (no toolkit/shim)     replaces README.md:126-149
  k8s-packages  pkgs.k8s.io v1.34 kubelet/kubeadm/kubectl (held)               README.md:159-187
  cluster       kubeadm init --config, kubeconfig, untaint, Flannel, Ready     README.md:191-243
  helm          pinned helm v3 release, sha256-verified (skipped if present)    README.md:249-255
  stack         amd-gpu-stack (helm, or kubectl apply of the rendered chart)   README.md:247-286
  validate      busybox (config 1) + hip-vector-add (config 2), wait + RESULT  README.md:288-335

``--dry-run --root DIR`` writes every file under DIR and records (does not
run) every command, which is what the CPU test tier checks.
"""
from __future__ import annotations

import dataclasses
import json
import os
import shlex
import shutil
import subprocess
import sys
import time
from typing import Callable, Optional, Sequence

from . import hostfiles as hf
from ..validate import isolation

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


@dataclasses.dataclass
class Context:
    root: str = "/"
    dry_run: bool = False
    upgrade: bool = False
    node_name: str = ""
    advertise_address: str = ""
    pod_cidr: str = hf.POD_CIDR
    kubernetes_version: str = hf.K8S_VERSION
    kubeconfig_home: str = os.path.expanduser("~")
    repo: str = REPO
    actions: list = dataclasses.field(default_factory=list)
    out: Callable[[str], None] = lambda s: print(s, file=sys.stderr)

    # ---- filesystem, relative to root ----
    def path(self, p: str) -> str:
        if self.root in ("", "/"):
            return p
        return os.path.join(self.root, p.lstrip("/"))

    def read(self, p: str) -> Optional[str]:
        try:
            with open(self.path(p)) as f:
                return f.read()
        except OSError:
            return None

    def exists(self, p: str) -> bool:
        return os.path.exists(self.path(p))

    def write(self, p: str, content: str, mode: int = 0o644) -> bool:
        """Write iff content differs. Returns True if the file changed."""
        if self.read(p) == content:
            return False
        full = self.path(p)
        os.makedirs(os.path.dirname(full), exist_ok=True)
        tmp = full + ".mxk8s-tmp"
        with open(tmp, "w") as f:
            f.write(content)
        os.chmod(tmp, mode)
        os.replace(tmp, full)
        self.actions.append(("write", p))
        return True

    # ---- commands ----
    def run(self, cmd: Sequence[str] | str, check: bool = True, capture: bool = False,
            env: Optional[dict] = None) -> subprocess.CompletedProcess:
        argv = shlex.split(cmd) if isinstance(cmd, str) else list(cmd)
        self.actions.append(("run", argv))
        if self.dry_run:
            return subprocess.CompletedProcess(argv, 0, "", "")
        self.out("+ " + " ".join(shlex.quote(a) for a in argv))
        return subprocess.run(argv, check=check, text=True,
                              capture_output=capture, env={**os.environ, **(env or {})})

    def have(self, tool: str) -> bool:
        return shutil.which(tool) is not None

    def commands(self) -> list[str]:
        return [" ".join(shlex.quote(a) for a in x[1]) for x in self.actions if x[0] == "run"]


class PhaseError(RuntimeError):
    pass


# ---------------------------------------------------------------------------
# phases
# ---------------------------------------------------------------------------

SUPPORTED_UBUNTU = ("22.04", "24.04", "24.10", "25.04", "25.10")


def preflight_report(ctx: Context) -> dict:
    """Host facts the preflight phase decides on (R00: the reference only
    states 'Ubuntu 25, NVIDIA GPU, root, internet' in prose, README.md:5-9)."""
    osr = {}
    for line in (ctx.read("/etc/os-release") or "").splitlines():
        k, _, v = line.partition("=")
        osr[k] = v.strip().strip('"')
    mem_kb = 0
    for line in (ctx.read("/proc/meminfo") or "").splitlines():
        if line.startswith("MemTotal:"):
            mem_kb = int(line.split()[1])
    try:
        st = os.statvfs(ctx.path("/var/lib") if ctx.exists("/var/lib") else ctx.path("/"))
        free_gb = st.f_bavail * st.f_frsize / 2 ** 30
    except OSError:
        free_gb = 0.0
    return {"os_id": osr.get("ID", ""), "os_version": osr.get("VERSION_ID", ""),
            "root": os.geteuid() == 0, "cpus": os.cpu_count() or 0,
            "mem_gib": round(mem_kb / 2 ** 20, 1), "free_disk_gib": round(free_gb, 1)}


def phase_preflight(ctx: Context) -> None:
    rep = preflight_report(ctx)
    if not rep["root"] and not ctx.dry_run:
        raise PhaseError("bootstrap needs root (sudo python3 -m mxk8s bootstrap); "
                         "use --dry-run --root DIR to inspect the plan")
    if rep["os_id"] != "ubuntu":
        ctx.out(f"WARNING: tested on Ubuntu {'/'.join(SUPPORTED_UBUNTU)}; found {rep['os_id'] or '?'}")
    elif rep["os_version"] not in SUPPORTED_UBUNTU:
        ctx.out(f"WARNING: Ubuntu {rep['os_version']} is untested "
                f"(tested: {', '.join(SUPPORTED_UBUNTU)})")
    if rep["mem_gib"] and rep["mem_gib"] < 64:
        ctx.out(f"WARNING: {rep['mem_gib']} GiB RAM; kubelet + an 8-GPU training pod want >= 64")
    if rep["free_disk_gib"] and rep["free_disk_gib"] < 50:
        ctx.out(f"WARNING: {rep['free_disk_gib']} GiB free under /var/lib (images need ~50)")
    ctx.out("preflight: " + json.dumps(rep))


def phase_prep(ctx: Context) -> None:
    if ctx.upgrade:
        ctx.run("apt-get update")
        ctx.run("apt-get upgrade -y")
    ctx.run("swapoff -a")
    fstab = ctx.read("/etc/fstab")
    if fstab is not None:
        ctx.write("/etc/fstab", hf.comment_swap(fstab))
    ctx.write("/etc/modules-load.d/k8s.conf", hf.modules_load_conf())
    ctx.run("modprobe overlay")
    ctx.run("modprobe br_netfilter")
    ctx.write("/etc/sysctl.d/k8s.conf", hf.sysctl_k8s_conf())
    ctx.write("/etc/sysctl.d/99-amd-gpu.conf", hf.sysctl_amd_gpu_conf())
    ctx.run("sysctl --system")


def driver_report(ctx: Context) -> dict:
    """Facts the driver gate decides on (also used by ``mxk8s doctor gpu``)."""
    from ..native import node
    rep = {"amdgpu_module": ctx.exists("/sys/module/amdgpu"),
           "kfd": ctx.exists("/dev/kfd"), "gpus": [], "errors": []}
    cmdline = ctx.read("/proc/cmdline") or ""
    rep["iommu_pt"] = "iommu=pt" in cmdline.split()
    try:
        gpus = node.enumerate_gpus("" if ctx.root in ("", "/") else ctx.root)
        rep["gpus"] = [g.to_dict() for g in gpus]
    except Exception as e:   # no KFD topology
        rep["errors"].append(str(e))
    rep["gfx950"] = sum(1 for g in rep["gpus"] if g["arch"] == "gfx950")
    return rep


def phase_driver_check(ctx: Context) -> None:
    rep = driver_report(ctx)
    problems = []
    if not rep["amdgpu_module"]:
        problems.append("amdgpu kernel module not loaded (install amdgpu-dkms + ROCm 7.x, reboot)")
    if not rep["kfd"]:
        problems.append("/dev/kfd missing (KFD not initialised)")
    if not rep["gpus"]:
        problems.append("no AMD GPUs in the KFD topology: " + "; ".join(rep["errors"]))
    if problems:
        # the reference's "Do not proceed" gate (README.md:84), made machine-checkable
        raise PhaseError("driver gate failed:\n  - " + "\n  - ".join(problems) +
                         "\nInstall the host driver, reboot, then re-run `mxk8s bootstrap` "
                         "(completed phases are skipped).")
    if not rep["iommu_pt"]:
        ctx.out("WARNING: kernel cmdline lacks iommu=pt (recommended for MI355X P2P/RCCL)")
    ctx.out(f"driver gate ok: {len(rep['gpus'])} GPU(s), {rep['gfx950']} gfx950")


def phase_runtime(ctx: Context) -> None:
    if not ctx.have("containerd") or ctx.dry_run:
        ctx.run("apt-get update")
        ctx.run("apt-get install -y apt-transport-https ca-certificates curl "
                "software-properties-common containerd")
    ctx.run("systemctl enable containerd")
    ctx.run("systemctl start containerd")
    ctx.run("containerd --version")
    current = ctx.read("/etc/containerd/config.toml")
    if not current:
        if ctx.dry_run or not ctx.have("containerd"):
            current = hf.minimal_containerd_config(2)
        else:
            current = ctx.run("containerd config default", capture=True).stdout
    ctx.write("/etc/containerd/config.toml", hf.configure_containerd(current))
    ctx.run("systemctl restart containerd")


def phase_cdi(ctx: Context) -> None:
    from ..native import node
    root = "" if ctx.root in ("", "/") else ctx.root
    spec = node.cdi_spec(root)
    ctx.write(hf.CDI_SPEC_PATH, json.dumps(spec, indent=2) + "\n")
    ctx.out(f"CDI spec: {len(spec['devices'])} device entries -> {hf.CDI_SPEC_PATH}")


def phase_k8s_packages(ctx: Context) -> None:
    ctx.run("apt-get update")
    ctx.run("apt-get install -y apt-transport-https ca-certificates curl gpg")
    ctx.run("mkdir -p -m 755 /etc/apt/keyrings")
    ctx.run(["bash", "-c",
             f"curl -fsSL https://pkgs.k8s.io/core:/stable:/{hf.k8s_minor(ctx.kubernetes_version)}/deb/Release.key | "
             "gpg --dearmor -o /etc/apt/keyrings/kubernetes-apt-keyring.gpg"])
    ctx.write("/etc/apt/sources.list.d/kubernetes.list", hf.kubernetes_apt_source(hf.k8s_minor(ctx.kubernetes_version)))
    ctx.run("apt-get update")
    ctx.run("apt-get install -y kubelet kubeadm kubectl")
    ctx.run("apt-mark hold kubelet kubeadm kubectl")
    ctx.run("systemctl enable --now kubelet")


def _kubectl(ctx: Context, *args: str, check: bool = True, capture: bool = False):
    return ctx.run(["kubectl", "--kubeconfig", "/etc/kubernetes/admin.conf", *args],
                   check=check, capture=capture)


def phase_cluster(ctx: Context) -> None:
    ctx.write("/etc/mxk8s/kubeadm-config.yaml",
              hf.kubeadm_config(ctx.node_name, ctx.advertise_address, ctx.kubernetes_version,
                                ctx.pod_cidr))
    if not ctx.exists("/etc/kubernetes/admin.conf") or ctx.dry_run:
        ctx.run(["kubeadm", "init", "--config", ctx.path("/etc/mxk8s/kubeadm-config.yaml")])
    home = ctx.kubeconfig_home
    ctx.run(["mkdir", "-p", f"{home}/.kube"])
    ctx.run(["cp", "-f", "/etc/kubernetes/admin.conf", f"{home}/.kube/config"])
    uid, gid = os.getuid(), os.getgid()
    ctx.run(["chown", f"{uid}:{gid}", f"{home}/.kube/config"])
    # single node: remove the control-plane taint (kubeadm config already sets
    # taints: [], this also fixes clusters initialised without our config)
    _kubectl(ctx, "taint", "nodes", "--all", "node-role.kubernetes.io/control-plane-", check=False)
    flannel = os.path.join(ctx.repo, "deploy", "cni", "kube-flannel.yaml")
    if ctx.pod_cidr != hf.POD_CIDR:
        # Flannel's net-conf must carry the same pod CIDR as kubeadm
        with open(flannel) as f:
            text = f.read().replace(f'"Network": "{hf.POD_CIDR}"', f'"Network": "{ctx.pod_cidr}"')
        ctx.write("/etc/mxk8s/kube-flannel.yaml", text)
        flannel = ctx.path("/etc/mxk8s/kube-flannel.yaml")
    _kubectl(ctx, "apply", "-f", flannel)
    _kubectl(ctx, "-n", "kube-flannel", "rollout", "status", "ds/kube-flannel-ds", "--timeout=300s")
    _kubectl(ctx, "wait", "node", "--all", "--for=condition=Ready", "--timeout=300s")


def phase_helm(ctx: Context) -> None:
    """Install the pinned helm release (the reference pipes get-helm-3 into
    bash, README.md:251-255).  The tarball is verified against the sha256 the
    release publishes next to it (or MXK8S_HELM_SHA256); offline hosts can
    point MXK8S_HELM_TARBALL at a copied tarball.  Without helm the stack phase
    applies the pre-rendered manifests instead, so a failure here only warns."""
    if ctx.have("helm") and not ctx.dry_run:
        ctx.out("helm already installed")
        return
    ver = hf.HELM_VERSION
    tgz = os.environ.get("MXK8S_HELM_TARBALL", f"/tmp/helm-{ver}-linux-amd64.tar.gz")
    url = f"https://get.helm.sh/helm-{ver}-linux-amd64.tar.gz"
    want = os.environ.get("MXK8S_HELM_SHA256", "")
    try:
        if not os.path.exists(tgz) or ctx.dry_run:
            ctx.run(["curl", "-fsSL", "-o", tgz, url])
        if not want:
            r = ctx.run(["curl", "-fsSL", url + ".sha256sum"], capture=True)
            want = (r.stdout or "").split()[0] if (r.stdout or "").strip() else ""
        if not ctx.dry_run:
            import hashlib
            with open(tgz, "rb") as f:
                got = hashlib.sha256(f.read()).hexdigest()
            if not want or got != want:
                raise PhaseError(f"helm tarball checksum mismatch: {got} != {want or '?'}")
        ctx.run(["tar", "-xzf", tgz, "-C", "/tmp", "linux-amd64/helm"])
        ctx.run(["install", "-m", "0755", "/tmp/linux-amd64/helm", "/usr/local/bin/helm"])
    except (subprocess.CalledProcessError, OSError, PhaseError) as e:
        ctx.out(f"WARNING: helm not installed ({e}); the stack phase will kubectl-apply "
                "deploy/amd-gpu-stack.yaml")


def phase_stack(ctx: Context) -> None:
    chart = os.path.join(ctx.repo, "charts", "amd-gpu-stack")
    if ctx.have("helm") and not ctx.dry_run:
        ctx.run(["helm", "upgrade", "--install", "amd-gpu-stack", chart, "-n", "amd-gpu",
                 "--create-namespace", "--set", "driver.enabled=false",
                 "--kubeconfig", "/etc/kubernetes/admin.conf"])
    else:
        _kubectl(ctx, "create", "namespace", "amd-gpu", check=False)
        _kubectl(ctx, "apply", "-f", os.path.join(ctx.repo, "deploy", "amd-gpu-stack.yaml"))
    _kubectl(ctx, "-n", "amd-gpu", "rollout", "status", "ds/amd-gpu-stack-device-plugin",
             "--timeout=300s")
    # capacity check (README.md:293-296): amd.com/gpu must be allocatable
    if not ctx.dry_run:
        deadline = time.time() + 120
        while True:
            r = _kubectl(ctx, "get", "nodes", "-o",
                         "jsonpath={.items[0].status.allocatable.amd\\.com/gpu}",
                         check=False, capture=True)
            if r.returncode == 0 and r.stdout.strip() not in ("", "0"):
                ctx.out(f"allocatable amd.com/gpu: {r.stdout.strip()}")
                break
            if time.time() > deadline:
                raise PhaseError("amd.com/gpu never became allocatable (see `mxk8s doctor gpu`)")
            time.sleep(3)


def phase_validate(ctx: Context) -> None:
    ex = os.path.join(ctx.repo, "deploy", "examples")
    for name, manifest in (("busybox-smoke", "busybox-smoke.yaml"),
                           ("hip-vector-add", "hip-vector-add.yaml")):
        _kubectl(ctx, "delete", "pod", name, "--ignore-not-found", check=False)
        _kubectl(ctx, "apply", "-f", os.path.join(ex, manifest))
        # instead of the reference's fixed `sleep 15` (README.md:326)
        _kubectl(ctx, "wait", f"pod/{name}", "--for=jsonpath={.status.phase}=Succeeded",
                 "--timeout=600s")
        r = _kubectl(ctx, "logs", f"pod/{name}", capture=True, check=False)
        if not ctx.dry_run and name == "hip-vector-add":
            # BASELINE.md:37: every RESULT line passes, the pod sees exactly
            # its one allocated gfx950 GPU (and only its render node)
            results = isolation.parse_results((r.stdout or "").splitlines())
            problems = isolation.check_results(results, gpus=1, arch="gfx950")
            if problems:
                raise PhaseError(f"{name}: " + "; ".join(problems))
            ctx.out(f"{name}: isolation ok ({len(results)} RESULT line(s))")


PHASES: list[tuple[str, Callable[[Context], None]]] = [
    ("preflight", phase_preflight),
    ("prep", phase_prep),
    ("driver-check", phase_driver_check),
    ("runtime", phase_runtime),
    ("cdi", phase_cdi),
    ("k8s-packages", phase_k8s_packages),
    ("cluster", phase_cluster),
    ("helm", phase_helm),
    ("stack", phase_stack),
    ("validate", phase_validate),
]
PHASE_NAMES = [n for n, _ in PHASES]


def completed(ctx: Context) -> list[str]:
    t = ctx.read(hf.PHASE_FILE)
    if not t:
        return []
    try:
        return list(json.loads(t).get("completed", []))
    except ValueError:
        return []


def mark(ctx: Context, name: str) -> None:
    done = completed(ctx)
    if name not in done:
        done.append(name)
    ctx.write(hf.PHASE_FILE, json.dumps({"completed": done, "updated": int(time.time())}) + "\n")


def run(ctx: Context, only: Optional[Sequence[str]] = None, resume: bool = True,
        until: Optional[str] = None) -> list[str]:
    """Run phases in order.  Returns the phases executed this call."""
    names = list(only) if only else PHASE_NAMES
    unknown = [n for n in names if n not in PHASE_NAMES]
    if unknown:
        raise ValueError(f"unknown phase(s) {unknown}; choose from {PHASE_NAMES}")
    done = set(completed(ctx)) if resume and not only else set()
    ran = []
    for name, fn in PHASES:
        if name not in names:
            continue
        if name in done:
            ctx.out(f"[mxk8s] phase {name}: already complete, skipping")
            continue
        ctx.out(f"[mxk8s] phase {name}")
        fn(ctx)
        mark(ctx, name)
        ran.append(name)
        if until and name == until:
            break
    return ran
