"""``mxk8s doctor {gpu,node,pod NAME}`` — the reference's troubleshooting section
(/root/reference/README.md:339-357) as executable decision trees.

README "GPU not detected" (:341-345): nvidia-smi -> device-plugin logs ->
grep nvidia config.toml.  Here: amdgpu/KFD/gfx950 gate -> CDI spec present
and current -> containerd CDI enabled -> plugin socket -> plugin pods
(label app=amd-gpu-device-plugin) -> allocatable amd.com/gpu == GPU count.
README "Node NotReady" (:347-351): kube-system pods, flannel pods, describe
node.  Here also swap/modules/sysctls.  README "Pod cannot access GPU"
(:353-357): request present? allocatable? operator running?  Here also the
scheduler's FailedScheduling reason (taints, insufficient amd.com/gpu).

Every check yields (name, status, detail, hint); status is ok / fail / skip
(kubectl or the host path not available).  Exit code 1 if any check fails;
the first failure's hint is printed last.
"""
from __future__ import annotations

import dataclasses
import json
import os
import shutil
import subprocess
from typing import Callable, Iterable, Optional

from ..bootstrap import hostfiles as hf


@dataclasses.dataclass
class Check:
    name: str
    status: str          # "ok" | "fail" | "skip"
    detail: str = ""
    hint: str = ""


class Host:
    """Filesystem + kubectl access, rooted (fake-able in tests)."""

    def __init__(self, root: str = "/", kubectl: Optional[Callable[..., tuple[int, str]]] = None):
        self.root = root
        self._kubectl = kubectl

    def path(self, p: str) -> str:
        return p if self.root in ("", "/") else os.path.join(self.root, p.lstrip("/"))

    def read(self, p: str) -> Optional[str]:
        try:
            with open(self.path(p)) as f:
                return f.read()
        except OSError:
            return None

    def exists(self, p: str) -> bool:
        return os.path.exists(self.path(p))

    def kubectl(self, *args: str) -> tuple[int, str]:
        if self._kubectl is not None:
            return self._kubectl(*args)
        if not shutil.which("kubectl"):
            return 127, "kubectl not found"
        p = subprocess.run(["kubectl", *args], capture_output=True, text=True, timeout=60)
        return p.returncode, p.stdout if p.returncode == 0 else p.stderr


def _sysfs_root(h: Host) -> str:
    return "" if h.root in ("", "/") else h.root


def check_gpu(h: Host) -> list[Check]:
    from ..native import node
    out = []
    amdgpu = h.exists("/sys/module/amdgpu")
    out.append(Check("amdgpu kernel module", "ok" if amdgpu else "fail",
                     "loaded" if amdgpu else "not loaded",
                     "install amdgpu-dkms + ROCm 7.x and reboot; then `mxk8s bootstrap --phase driver-check`"))
    kfd = h.exists("/dev/kfd")
    out.append(Check("/dev/kfd", "ok" if kfd else "fail", "present" if kfd else "missing",
                     "KFD not initialised: check `dmesg | grep -i kfd`"))
    try:
        gpus = node.enumerate_gpus(_sysfs_root(h))
    except Exception as e:
        gpus = []
        out.append(Check("GPU enumeration (KFD topology)", "fail", str(e),
                         "no KFD topology: the amdgpu driver is not bound to any GPU"))
    else:
        archs = sorted({g.arch for g in gpus})
        ok = bool(gpus) and archs == ["gfx950"]
        out.append(Check("GPU enumeration (KFD topology)", "ok" if ok else "fail",
                         f"{len(gpus)} GPU(s), arch {','.join(archs) or '-'}",
                         "expected gfx950 (MI355X) GPUs"))
        missing = [g.render_path for g in gpus if not h.exists(g.render_path)]
        out.append(Check("render nodes", "fail" if missing else "ok",
                         ("missing " + ", ".join(missing)) if missing else f"{len(gpus)} present",
                         "device nodes missing: GPU reset/unbound? check dmesg"))
    spec_txt = h.read(hf.CDI_SPEC_PATH)
    if spec_txt is None:
        out.append(Check("CDI spec", "fail", f"{hf.CDI_SPEC_PATH} missing",
                         "run `mxk8s bootstrap --phase cdi` (or bin/mx-cdi-gen --output ...)"))
    else:
        try:
            cur = json.loads(spec_txt)
            want = node.cdi_spec(_sysfs_root(h)) if gpus else None
            if want is not None and cur != want:
                out.append(Check("CDI spec", "fail", "stale (does not match current GPUs)",
                                 "regenerate: `mxk8s cdi --output /etc/cdi/amd.com-gpu.json`"))
            else:
                out.append(Check("CDI spec", "ok", f"{len(cur.get('devices', []))} device entries"))
        except ValueError as e:
            out.append(Check("CDI spec", "fail", f"invalid JSON: {e}", "regenerate the spec"))
    cfg = h.read("/etc/containerd/config.toml")
    if cfg is None:
        out.append(Check("containerd CDI", "skip", "no /etc/containerd/config.toml"))
    else:
        cdi_on = "enable_cdi = true" in cfg
        sysd = "SystemdCgroup = true" in cfg
        out.append(Check("containerd CDI", "ok" if cdi_on else "fail",
                         "enable_cdi = true" if cdi_on else "CDI not enabled",
                         "`mxk8s bootstrap --phase runtime` (containerd 2.x has CDI on by default)"))
        out.append(Check("containerd SystemdCgroup", "ok" if sysd else "fail",
                         "true" if sysd else "false", "set SystemdCgroup = true (README.md:123)"))
    # node-validator markers (operator-validator counterpart): which layer of
    # the chain last failed, for the running boot + driver instance
    from ..validate import node as vnode
    vdir = h.path(vnode.validations_dir("/var/lib/mxk8s"))
    if not os.path.isdir(vdir):
        out.append(Check("node validation", "skip", "no /var/lib/mxk8s/validations (validator not deployed)"))
    else:
        st = vnode.status(os.path.dirname(vdir), _sysfs_root(h))
        bad = [k for k, ok in st.items() if not ok]
        detail = ", ".join(f"{k}={'ready' if ok else 'NOT ready'}" for k, ok in st.items())
        hint = (f"first failing step: {bad[0]}: `kubectl -n amd-gpu logs -l app=amd-gpu-node-validator "
                f"-c {bad[0]}-validation`" if bad else "")
        out.append(Check("node validation", "fail" if bad else "ok", detail, hint))
    sock = h.exists("/var/lib/kubelet/device-plugins/amd-gpu.sock")
    out.append(Check("device plugin socket", "ok" if sock else "fail",
                     "registered socket present" if sock else "amd-gpu.sock missing",
                     "plugin not running: `kubectl -n amd-gpu logs -l app=amd-gpu-device-plugin`"))
    rc, txt = h.kubectl("get", "pods", "-A", "-l", "app=amd-gpu-device-plugin", "-o", "json")
    if rc == 127:
        out.append(Check("device plugin pods", "skip", txt))
    elif rc != 0:
        out.append(Check("device plugin pods", "fail", txt.strip()[:200], "is the API server up?"))
    else:
        pods = json.loads(txt).get("items", [])
        running = [p for p in pods if p.get("status", {}).get("phase") == "Running"]
        out.append(Check("device plugin pods", "ok" if running else "fail",
                         f"{len(running)}/{len(pods)} running",
                         "`helm install amd-gpu-stack ./charts/amd-gpu-stack -n amd-gpu --create-namespace`"))
        resource, replicas = plugin_sharing(pods)
        rc, txt = h.kubectl("get", "nodes", "-o", "json")
        if rc == 0:
            items = json.loads(txt).get("items", [])
            alloc = sum(int(n.get("status", {}).get("allocatable", {}).get(resource, 0))
                        for n in items)
            want_n = len(gpus) * replicas
            good = alloc == want_n and want_n > 0
            shared = f" ({len(gpus)} GPUs x {replicas} time-sliced replicas)" if replicas > 1 else ""
            out.append(Check(f"allocatable {resource}", "ok" if good else "fail",
                             f"{alloc} allocatable, {want_n} expected{shared}",
                             f"unhealthy devices? `kubectl describe node | grep {resource}`"))
    return out


def plugin_sharing(pods: list) -> tuple[str, int]:
    """(advertised resource name, replicas per GPU) from the running device
    plugin's arguments: time-slicing advertises replicas x GPUs, under
    ``<resource>.shared`` when renaming is on."""
    resource, replicas, rename = "amd.com/gpu", 1, False
    for p in pods:
        for c in p.get("spec", {}).get("containers", []):
            for a in c.get("args", []) or []:
                k, _, v = a.partition("=")
                if k == "--resource-name" and v:
                    resource = v
                elif k == "--replicas" and v.isdigit():
                    replicas = max(1, int(v))
                elif k == "--rename-shared":
                    rename = v.lower() in ("1", "true", "yes", "on")
        break
    if replicas > 1 and rename and not resource.endswith(".shared"):
        resource += ".shared"
    return resource, replicas


def check_node(h: Host) -> list[Check]:
    out = []
    swaps = (h.read("/proc/swaps") or "").strip().splitlines()[1:]
    out.append(Check("swap off", "fail" if swaps else "ok", f"{len(swaps)} active swap device(s)",
                     "swapoff -a and comment swap in /etc/fstab (README.md:28-29)"))
    mods = h.read("/proc/modules")
    if mods is None:
        out.append(Check("kernel modules", "skip", "/proc/modules unreadable"))
    else:
        names = {l.split()[0] for l in mods.splitlines() if l.strip()}
        miss = [m for m in ("overlay", "br_netfilter") if m not in names]
        out.append(Check("kernel modules", "fail" if miss else "ok",
                         ("missing " + ",".join(miss)) if miss else "overlay, br_netfilter",
                         "modprobe overlay br_netfilter (README.md:37-43)"))
    for key, want in (("net/ipv4/ip_forward", "1"), ("net/bridge/bridge-nf-call-iptables", "1")):
        v = h.read(f"/proc/sys/{key}")
        if v is None:
            out.append(Check(f"sysctl {key}", "skip", "unreadable"))
        else:
            out.append(Check(f"sysctl {key}", "ok" if v.strip() == want else "fail", v.strip(),
                             "sysctl --system after writing /etc/sysctl.d/k8s.conf"))
    rc, txt = h.kubectl("get", "nodes", "-o", "json")
    if rc == 127:
        out.append(Check("node Ready", "skip", txt))
        return out
    if rc != 0:
        out.append(Check("node Ready", "fail", txt.strip()[:200], "kubelet running? `systemctl status kubelet`"))
        return out
    for n in json.loads(txt).get("items", []):
        conds = {c["type"]: c for c in n.get("status", {}).get("conditions", [])}
        ready = conds.get("Ready", {}).get("status") == "True"
        out.append(Check(f"node {n['metadata']['name']} Ready", "ok" if ready else "fail",
                         conds.get("Ready", {}).get("message", ""),
                         "CNI not ready? `kubectl get pods -n kube-flannel` (README.md:347-351)"))
        taints = [t for t in n.get("spec", {}).get("taints", []) or []
                  if t.get("key") == "node-role.kubernetes.io/control-plane"]
        out.append(Check("control-plane taint", "fail" if taints else "ok",
                         "present" if taints else "removed",
                         "kubectl taint nodes --all node-role.kubernetes.io/control-plane-"))
    for ns in ("kube-system", "kube-flannel"):
        rc, txt = h.kubectl("get", "pods", "-n", ns, "-o", "json")
        if rc != 0:
            continue
        pods = json.loads(txt).get("items", [])
        bad = [p["metadata"]["name"] for p in pods
               if p.get("status", {}).get("phase") not in ("Running", "Succeeded")]
        out.append(Check(f"{ns} pods", "fail" if bad else "ok",
                         ("not running: " + ",".join(bad)) if bad else f"{len(pods)} running",
                         f"kubectl -n {ns} describe pod <name>"))
    return out


def check_pod(h: Host, name: str, namespace: str = "default") -> list[Check]:
    out = []
    rc, txt = h.kubectl("get", "pod", name, "-n", namespace, "-o", "json")
    if rc == 127:
        return [Check("pod", "skip", txt)]
    if rc != 0:
        return [Check("pod exists", "fail", txt.strip()[:200], f"kubectl get pod {name} -n {namespace}")]
    pod = json.loads(txt)
    req = 0
    for c in pod.get("spec", {}).get("containers", []):
        req += int(c.get("resources", {}).get("limits", {}).get("amd.com/gpu", 0))
    out.append(Check("requests amd.com/gpu", "ok" if req else "fail", f"limit {req}",
                     "add resources.limits: {amd.com/gpu: N} (README.md:355)"))
    tol = [t for t in pod.get("spec", {}).get("tolerations", []) or []
           if t.get("key") in ("node-role.kubernetes.io/control-plane",) or t.get("operator") == "Exists" and not t.get("key")]
    phase = pod.get("status", {}).get("phase", "")
    out.append(Check("pod phase", "ok" if phase in ("Running", "Succeeded") else "fail", phase,
                     "see scheduling events below"))
    for c in pod.get("status", {}).get("conditions", []) or []:
        if c.get("type") == "PodScheduled" and c.get("status") != "True":
            msg = c.get("message", "")
            hint = "no node has enough allocatable amd.com/gpu (`mxk8s doctor gpu`)"
            if "taint" in msg:
                hint = ("the control-plane taint blocks it: add a toleration or "
                        "`kubectl taint nodes --all node-role.kubernetes.io/control-plane-`")
            out.append(Check("scheduling", "fail", msg, hint))
    out.append(Check("control-plane toleration", "ok" if tol else "skip",
                     "present" if tol else "absent (fine once the node is untainted)"))
    return out


def run(checks: Iterable[Check], out=print) -> int:
    checks = list(checks)
    first_fail = None
    for c in checks:
        mark = {"ok": "OK  ", "fail": "FAIL", "skip": "SKIP"}[c.status]
        out(f"[{mark}] {c.name}: {c.detail}")
        if c.status == "fail" and first_fail is None:
            first_fail = c
    if first_fail:
        out(f"\nfirst failure: {first_fail.name}\n  fix: {first_fail.hint}")
        return 1
    return 0
