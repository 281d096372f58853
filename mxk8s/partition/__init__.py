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
     single-node cluster has nowhere to move them);
  5. write the memory mode, then the compute mode, to every device; wait for
     the KFD topology to show devices x partitions GPUs; state ``success`` or
     ``failed`` with the reason in annotation ``amd.com/gpu.partition.config.message``.

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


class PartitionManager:
    def __init__(self, client, node_name: str, sysfs_root: str = "",
                 profiles: Optional[dict] = None,
                 busy: Optional[Callable[[], list[str]]] = None,
                 settle_timeout: float = 120.0, poll: float = 1.0):
        self.client = client
        self.node_name = node_name
        self.root = sysfs_root
        self.profiles = {k: {"compute": v["compute"].upper(), "memory": v["memory"].upper()}
                         for k, v in (profiles or DEFAULT_PROFILES).items()}
        self.busy = busy or (lambda: [])
        self.settle_timeout = settle_timeout
        self.poll = poll
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
            return Result("success", f"{name}: {prof['compute']}/{prof['memory']} on "
                                     f"{len(bdfs)} device(s), {len(gpus)} GPU partitions")
        users = self.busy()
        if users:
            return Result("pending", f"waiting for {len(users)} GPU workload(s) to finish: "
                                     + ", ".join(users[:5]))
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
                return Result("failed", f"{name}: driver shows {n} GPU(s), expected {want} "
                                        f"after {self.settle_timeout:.0f} s", applied=True)
            time.sleep(self.poll)


def pod_resources_users(socket_path: Optional[str], resource: str = "amd.com/gpu") -> list[str]:
    """Containers holding GPUs (any amd.com/gpu* resource) per the kubelet."""
    if not socket_path or not os.path.exists(socket_path):
        return []
    from ..exporter.podresources import ListPodResourcesRequest, ListPodResourcesResponse, LIST_METHOD
    import grpc
    with grpc.insecure_channel("unix:" + socket_path) as ch:
        call = ch.unary_unary(LIST_METHOD, request_serializer=ListPodResourcesRequest.SerializeToString,
                              response_deserializer=ListPodResourcesResponse.FromString)
        resp = call(ListPodResourcesRequest(), timeout=5)
    out = []
    for pr in resp.pod_resources:
        for c in pr.containers:
            if any(d.resource_name.startswith(resource) and d.device_ids for d in c.devices):
                out.append(f"{pr.namespace}/{pr.name}/{c.name}")
    return out


def smi_users() -> list[str]:
    ok, _ = node.smi_open()
    if not ok:
        return []
    out = []
    for i in range(max(0, node.smi_count())):
        out += [f"pid {p.pid} ({p.name})" for p in node.smi_processes(i)]
    return out
