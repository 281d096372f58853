"""GPU partition manager — the MI355X counterpart of the GPU Operator's MIG
manager (an operand of the chart the reference installs at
/root/reference/README.md:269-271).

NVIDIA's MIG manager watches the node label ``nvidia.com/mig.config``, applies
the named MIG layout with nvidia-smi and reports ``nvidia.com/mig.config.state``.
An MI355X has no MIG; it has two partition knobs exposed by amdgpu per PCI
device in sysfs:

  * compute partitioning  ``current_compute_partition``  SPX | DPX | QPX | CPX
    (1 / 2 / 4 / 8 partitions of the 8 XCDs, each its own KFD node + render
    node, so each schedulable as its own device),
  * memory partitioning   ``current_memory_partition``   NPS1 | NPS2 (the HBM
    stacks interleaved over the whole device or split per half).

Reconcile loop (one node, one DaemonSet pod):

  1. desired profile = node label ``amd.com/gpu.partition.config`` (a name from
     ``profiles``, e.g. ``cpx-nps2``); no label: nothing to do;
  2. the profile must be one every device lists in
     ``available_{compute,memory}_partition`` — else state ``failed``;
  3. already there: state ``success``;
  4. GPUs in use (the kubelet PodResources API shows ``amd.com/gpu*``
     allocations, or amd-smi lists processes): state ``pending`` and retry —
     no workload is ever yanked (the MIG manager evicts GPU clients; a
     single-node cluster has nowhere to move them).  The check fails CLOSED:
     a probe that cannot answer (socket missing, amd-smi not loadable) is
     ``pending`` too, never "idle";
  5. drain: write ``<state_dir>/partition-drain`` (hostPath /var/lib/mxk8s,
     shared with the device plugin), which makes the plugin advertise every
     device Unhealthy ("partition change in progress") and acknowledge in
     ``partition-drain.ack``; so no pod can be admitted while sysfs changes.
     Then the busy check runs AGAIN (a pod admitted between the first check
     and the drain is caught) — still busy: ``pending``, drain lifted;
  6. write the memory mode, then the compute mode, to every device; wait for
     the KFD topology to show devices x partitions GPUs: ``success`` (drain
     lifted), or — amdgpu took the modes (sysfs reads them back) but did not
     re-enumerate, as an NPS change needs a driver reload — ``pending-reboot``
     (drain kept until the node comes back in the requested layout), or
     ``failed`` when the driver rejected a mode; the reason goes to annotation
     ``amd.com/gpu.partition.config.message``.

The device plugin's reconciliation (``mxk8s.deviceplugin.plugin``) notices
the new GPU set and re-advertises (as ``amd.com/gpu`` or, with mixed naming,
``amd.com/gpu-cpx``); the labeller publishes the modes.
"""
from __future__ import annotations

import dataclasses
import logging
import os
import time
from typing import Callable, Optional

from ..native import node

log = logging.getLogger("mxk8s.partition")

CONFIG_LABEL = "amd.com/gpu.partition.config"
STATE_LABEL = "amd.com/gpu.partition.config.state"
MESSAGE_ANNOTATION = "amd.com/gpu.partition.config.message"
PARTS = {"SPX": 1, "DPX": 2, "QPX": 4, "CPX": 8}

DEFAULT_PROFILES = {
    "spx-nps1": {"compute": "SPX", "memory": "NPS1"},
    "dpx-nps1": {"compute": "DPX", "memory": "NPS1"},
    "qpx-nps1": {"compute": "QPX", "memory": "NPS1"},
    "cpx-nps1": {"compute": "CPX", "memory": "NPS1"},
    "dpx-nps2": {"compute": "DPX", "memory": "NPS2"},
    "cpx-nps2": {"compute": "CPX", "memory": "NPS2"},
}


@dataclasses.dataclass
class Result:
    state: str                  # success | pending | failed | none
    message: str
    applied: bool = False


def _pci(root: str, bdf: str, name: str) -> str:
    return os.path.join(root or "/", "sys/bus/pci/devices", bdf, name)


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def physical_devices(gpus: list[node.GpuInfo]) -> list[str]:
    """BDFs of the PCI devices (partition 0 of each), in GPU order."""
    return [g.bdf for g in gpus if g.partition == 0]


def current_modes(root: str, bdfs: list[str]) -> dict:
    out = {}
    for b in bdfs:
        out[b] = {"compute": (_read(_pci(root, b, "current_compute_partition")) or "").upper(),
                  "memory": (_read(_pci(root, b, "current_memory_partition")) or "").upper()}
    return out


def available_modes(root: str, bdf: str, kind: str) -> set[str]:
    text = _read(_pci(root, bdf, f"available_{kind}_partition")) or ""
    return {t.strip().upper() for t in text.replace(",", " ").split() if t.strip()}


DRAIN_FILE = "partition-drain"
DRAIN_ACK_FILE = "partition-drain.ack"
DRAIN_REASON = "partition change in progress"


def boot_id(path: str = "/proc/sys/kernel/random/boot_id") -> str:
    return (_read(path) or "unknown").strip()


def read_drain(state_dir: Optional[str], boot: Optional[str] = None) -> Optional[str]:
    """The active drain token in ``state_dir`` (None: no drain).  A drain
    written in an earlier boot is void: the node came back from the reboot
    a pending-reboot layout asked for, so the plugin must serve again even if
    no manager runs to lift it."""
    if not state_dir:
        return None
    text = _read(os.path.join(state_dir, DRAIN_FILE))
    if not text:
        return None
    token, _, drain_boot = text.partition(" ")
    if drain_boot.strip() and drain_boot.strip() != (boot or boot_id()):
        return None
    return token


def _write_atomic(path: str, text: str) -> None:
    tmp = path + ".tmp"
    with open(tmp, "w") as f:
        f.write(text)
    os.replace(tmp, path)


class PartitionManager:
    def __init__(self, client, node_name: str, sysfs_root: str = "",
                 profiles: Optional[dict] = None,
                 busy: Optional[Callable[[], Optional[list[str]]]] = None,
                 settle_timeout: float = 120.0, poll: float = 1.0,
                 state_dir: Optional[str] = None, drain_timeout: float = 30.0,
                 plugin_fresh_s: float = 60.0, boot: Optional[str] = None):
        self.client = client
        self.node_name = node_name
        self.root = sysfs_root
        self.profiles = {k: {"compute": v["compute"].upper(), "memory": v["memory"].upper()}
                         for k, v in (profiles or DEFAULT_PROFILES).items()}
        # busy() -> users, or None when it cannot tell (then: never repartition)
        self.busy = busy or (lambda: [])
        self.settle_timeout = settle_timeout
        self.poll = poll
        self.state_dir = state_dir
        self.drain_timeout = drain_timeout
        self.plugin_fresh_s = plugin_fresh_s
        self.boot = boot or boot_id()
        self._last_state: Optional[tuple] = None

    # ---------------------------------------------------------------- k8s
    def desired(self) -> Optional[str]:
        labels = self.client.get_node(self.node_name).get("metadata", {}).get("labels", {}) or {}
        return labels.get(CONFIG_LABEL)

    def report(self, res: Result) -> None:
        key = (res.state, res.message)
        if key == self._last_state:
            return
        self._last_state = key
        self.client.merge_patch(f"/api/v1/nodes/{self.node_name}", {
            "metadata": {"labels": {STATE_LABEL: res.state},
                         "annotations": {MESSAGE_ANNOTATION: res.message}}})
        lvl = logging.WARNING if res.state == "failed" else logging.INFO
        log.log(lvl, "partition config %s: %s", res.state, res.message,
                extra={"event": "partition_" + res.state, "reason": res.message})

    # ---------------------------------------------------------------- core
    def reconcile_once(self) -> Result:
        want_name = self.desired()
        if not want_name:
            return Result("none", "no amd.com/gpu.partition.config label")
        res = self.apply(want_name)
        self.report(res)
        return res

    def apply(self, name: str) -> Result:
        prof = self.profiles.get(name)
        if prof is None:
            return Result("failed", f"unknown partition profile {name!r} "
                                    f"(known: {', '.join(sorted(self.profiles))})")
        gpus = node.enumerate_gpus(self.root)
        bdfs = physical_devices(gpus)
        if not bdfs:
            return Result("failed", "no AMD GPU found")
        for b in bdfs:
            for kind in ("compute", "memory"):
                avail = available_modes(self.root, b, kind)
                if not avail:
                    return Result("failed", f"{b}: amdgpu exposes no {kind} partitioning")
                if prof[kind] not in avail:
                    return Result("failed", f"{b}: {kind} mode {prof[kind]} not in "
                                            f"{sorted(avail)}")
        cur = current_modes(self.root, bdfs)
        todo = [b for b in bdfs if cur[b] != prof]
        if not todo:
            self._set_drain(None)     # e.g. back from the reboot a pending-reboot asked for
            return Result("success", f"{name}: {prof['compute']}/{prof['memory']} on "
                                     f"{len(bdfs)} device(s), {len(gpus)} GPU partitions")
        users = self.busy()
        if users is None:
            return Result("pending", "cannot verify that the GPUs are idle (pod-resources or "
                                     "amd-smi probe unavailable); not repartitioning")
        if users:
            return Result("pending", f"waiting for {len(users)} GPU workload(s) to finish: "
                                     + ", ".join(users[:5]))
        # withdraw the devices from the scheduler before touching sysfs
        token = f"{name}@{int(time.time() * 1000)}"
        keep_drain = False
        self._set_drain(token)
        try:
            if not self._wait_drain_ack(token):
                return Result("pending", "the device plugin did not acknowledge the drain within "
                                         f"{self.drain_timeout:.0f} s; not repartitioning")
            users = self.busy()          # admitted between the first check and the drain?
            if users is None or users:
                return Result("pending", "GPU workload(s) started before the drain took effect: "
                                         + (", ".join(users[:5]) if users else "probe unavailable"))
            res = self._write_and_settle(name, prof, bdfs, todo, cur)
            keep_drain = res.state == "pending-reboot"
            return res
        finally:
            if not keep_drain:
                self._set_drain(None)

    def _write_and_settle(self, name, prof, bdfs, todo, cur) -> Result:
        # memory first (a compute partition is carved out of the memory layout)
        for kind in ("memory", "compute"):
            for b in todo:
                if cur[b][kind] == prof[kind]:
                    continue
                try:
                    with open(_pci(self.root, b, f"current_{kind}_partition"), "w") as f:
                        f.write(prof[kind] + "\n")
                except OSError as e:
                    return Result("failed", f"{b}: writing {kind} mode {prof[kind]}: {e}",
                                  applied=True)
        want = len(bdfs) * PARTS[prof["compute"]]
        deadline = time.monotonic() + self.settle_timeout
        while True:
            try:
                n = len(node.enumerate_gpus(self.root))
            except RuntimeError:
                n = -1
            now = current_modes(self.root, bdfs)
            if n == want and all(now[b] == prof for b in bdfs):
                return Result("success", f"{name}: {prof['compute']}/{prof['memory']} on "
                                         f"{len(bdfs)} device(s), {n} GPU partitions", applied=True)
            if time.monotonic() >= deadline:
                if all(now[b] == prof for b in bdfs):
                    # amdgpu took the modes but did not re-enumerate in place (an
                    # NPS change needs a driver reload): not a failure of the request
                    return Result("pending-reboot",
                                  f"{name}: amdgpu reports {prof['compute']}/{prof['memory']} but "
                                  f"the KFD topology shows {n} GPU(s), expected {want} after "
                                  f"{self.settle_timeout:.0f} s: reload amdgpu or reboot the node "
                                  f"(devices stay drained until then)", applied=True)
                bad = [b for b in bdfs if now[b] != prof]
                return Result("failed", f"{name}: driver shows {n} GPU(s), expected {want}; "
                                        f"{len(bad)} device(s) read back other modes "
                                        f"({bad[0]}: {now[bad[0]]['compute']}/{now[bad[0]]['memory']}) "
                                        f"after {self.settle_timeout:.0f} s", applied=True)
            time.sleep(self.poll)

    # ------------------------------------------------------------- drain
    def _set_drain(self, token: Optional[str]) -> None:
        if not self.state_dir:
            return
        path = os.path.join(self.state_dir, DRAIN_FILE)
        if token is None:
            for p in (path, os.path.join(self.state_dir, DRAIN_ACK_FILE)):
                try:
                    os.unlink(p)
                except FileNotFoundError:
                    pass
            return
        os.makedirs(self.state_dir, exist_ok=True)
        _write_atomic(path, f"{token} {self.boot}\n")

    def _plugin_running(self) -> bool:
        """The device plugin refreshes <state_dir>/health.json every pass."""
        try:
            age = time.time() - os.stat(os.path.join(self.state_dir, "health.json")).st_mtime
        except (OSError, TypeError):
            return False
        return age <= self.plugin_fresh_s

    def _wait_drain_ack(self, token: str) -> bool:
        if not self.state_dir or not self._plugin_running():
            return True               # no plugin serving: nothing can be admitted
        deadline = time.monotonic() + self.drain_timeout
        while time.monotonic() < deadline:
            if (_read(os.path.join(self.state_dir, DRAIN_ACK_FILE)) or "") == token:
                return True
            time.sleep(min(self.poll, 0.1))
        return False


def pod_resources_users(socket_path: Optional[str],
                        resource: str = "amd.com/gpu") -> Optional[list[str]]:
    """Containers holding GPUs (any amd.com/gpu* resource) per the kubelet;
    None when the pod-resources API cannot be asked (fail closed)."""
    if not socket_path or not os.path.exists(socket_path):
        return None
    from ..exporter.podresources import ListPodResourcesRequest, ListPodResourcesResponse, LIST_METHOD
    import grpc
    try:
        with grpc.insecure_channel("unix:" + socket_path) as ch:
            call = ch.unary_unary(LIST_METHOD,
                                  request_serializer=ListPodResourcesRequest.SerializeToString,
                                  response_deserializer=ListPodResourcesResponse.FromString)
            resp = call(ListPodResourcesRequest(), timeout=5)
    except grpc.RpcError as e:
        log.warning("pod-resources probe failed: %s", e)
        return None
    out = []
    for pr in resp.pod_resources:
        for c in pr.containers:
            if any(d.resource_name.startswith(resource) and d.device_ids for d in c.devices):
                out.append(f"{pr.namespace}/{pr.name}/{c.name}")
    return out


def smi_users() -> Optional[list[str]]:
    """Processes with a context on any GPU per amd-smi; None when amd-smi
    cannot be opened (fail closed)."""
    ok, _ = node.smi_open()
    if not ok:
        return None
    try:
        out = []
        for i in range(max(0, node.smi_count())):
            out += [f"pid {p.pid} ({p.name})" for p in node.smi_processes(i)]
        return out
    finally:
        node.smi_close()


def combined_busy(*probes: Callable[[], Optional[list[str]]]) -> Callable[[], Optional[list[str]]]:
    """busy() over several probes: None if any probe cannot answer."""
    def busy():
        users: list[str] = []
        for probe in probes:
            got = probe()
            if got is None:
                return None
            users += got
        return users
    return busy
